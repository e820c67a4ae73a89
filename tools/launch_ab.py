"""Interleaved A/B of the exclusive trace launches of teapot pass 0 (one pass context, as bench.py's
exclusive_pass) across librtamd.so variants: per variant, best of 3 runs of the per-bounce trace launch
spans (rt_renderer_launch_profile), bounces 0, 1, 2 and the rest summed, plus the pass's kernel time.
    python tools/launch_ab.py ROUNDS name1 name2 ...   (name: variant[@VAR=v,...], as tools/ab.py)
Run on the GPU box after tools/variants.sh here."""
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
os.environ["RTAMD_INFLIGHT"] = "1"
sys.path[:0] = [os.path.join(%(repo)r, "cuda-raytracer_amd"), os.path.join(%(repo)r, "tools")]
import make_envmap, rtamd
make_envmap.ensure_envmap(os.path.join(%(repo)r, "assets", "teapot", "textures", "envmap.pfm"))
scene = rtamd.Scene(os.path.join(rtamd.ASSETS, %(scene)r), image=%(image)r)
r = rtamd.Renderer(scene, sort=True)
r.set_event_timing(True)
r.run(0, 1)
best = None
for k in range(3):
    st = r.run(0, 1)
    prof = r.launch_profile()
    rec = {"kernel_ms": st["kernel_ms"], "launch_ms": [p[0] for p in prof], "live": [p[1] for p in prof]}
    if best is None or rec["kernel_ms"] < best["kernel_ms"]:
        best = rec
r.close()
print(json.dumps(best))
"""


def main():
    rounds, names = int(sys.argv[1]), sys.argv[2:]
    scene = os.environ.get("LAB_SCENE", "teapot.scene")
    image = tuple(int(x) for x in os.environ.get("LAB_IMAGE", "1920,1080,2048,16").split(","))
    res = {n: [] for n in names}
    for r in range(rounds):
        for n in names:
            base, _, extra_env = n.partition("@")
            lib = os.path.join(REPO, "cuda-raytracer_amd", "build_var", base, "librtamd.so")
            if base == "default":
                lib = os.path.join(REPO, "cuda-raytracer_amd", "build", "librtamd.so")
            env = dict(os.environ, RTAMD_LIB=lib)
            for kv in filter(None, extra_env.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            out = subprocess.run([sys.executable, "-c", CHILD % {"repo": REPO, "scene": scene, "image": image}],
                                 cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print("variant %s failed rc=%d: %s" % (n, out.returncode, out.stderr[-2000:]), flush=True)
                sys.exit(1)
            rec = json.loads(out.stdout.strip().splitlines()[-1])
            lm = rec["launch_ms"]
            row = (lm[0], lm[1], lm[2], sum(lm[3:]), sum(lm), rec["kernel_ms"])
            res[n].append(row)
            print("round %d %-28s b0 %.3f b1 %.3f b2 %.3f rest %.3f trace %.3f kernels %.3f" % ((r, n) + row),
                  flush=True)
    print("summary (medians: bounce 0, 1, 2, rest, trace sum, pass kernels ms):")
    for n in names:
        cols = list(zip(*res[n]))
        print("%-28s %s" % (n, " ".join("%.3f" % statistics.median(c) for c in cols)))


if __name__ == "__main__":
    main()
