"""What would batching the tails of k passes into one launch sequence buy?  Emulated by ONE teapot pass over k times
the pixels (20 spp, sqrt(k)-scaled 1080p image: k times the rays, one stream, one hardware queue busy), whose tail
(bounces 2-15) is compared with k real passes started together (tools/tail_probe.py, RTAMD_TIMELINE).
    python tools/batch_tail_probe.py [k ...]"""
import math
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ks = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 6]
CHILD = r'''
import os, sys
sys.path[:0] = [os.path.join(%(repo)r, "cuda-raytracer_amd"), os.path.join(%(repo)r, "tools")]
os.environ["RTAMD_TIMELINE"] = "1"
import make_envmap, rtamd
make_envmap.ensure_envmap(os.path.join(%(repo)r, "assets", "teapot", "textures", "envmap.pfm"))
scene = rtamd.Scene(os.path.join(rtamd.ASSETS, "teapot.scene"), image=(%(w)d, %(h)d, 20, 16))
r = rtamd.Renderer(scene, sort=True)
r.set_event_timing(True)
for rep in range(3):
    r.run(0, 1)
r.close()
'''
for k in ks:
    w, h = round(1920 * math.sqrt(k)), round(1080 * math.sqrt(k))
    # one process per size (each renderer sizes its contexts for its image); the timeline goes to stderr
    p = subprocess.run([sys.executable, "-c", CHILD % {"repo": REPO, "w": w, "h": h}], capture_output=True, text=True,
                       timeout=600)
    if p.returncode:
        sys.exit(p.stderr[-2000:])
    lines = [l for l in p.stderr.splitlines() if l.startswith("timeline pass")]
    best = None
    for l in lines:                      # "timeline pass 0: b0 b1 b2 | end"
        a = l.split(":")[1].replace("|", " ").split()
        b0, b1, b2, e = map(float, a)
        if best is None or e < best[3]:
            best = (b0, b1, b2, e)
    b0, b1, b2, e = best
    print("k=%d  %dx%d (%.1f M rays): heavy %.2f ms, tail %.2f ms, pass %.2f ms (best of %d)"
          % (k, w, h, w * h * 20 / 1e6, b2 - b0, e - b2, e - b0, len(lines)), flush=True)
