"""Do concurrent tails slow each other inside the trace launches or between them?  Runs k teapot passes together
(event timing on) and prints pass 0's trace-launch spans per bounce (rt_renderer_launch_profile, device wall
clock) next to the bounce starts and end of every pass (RTAMD_TIMELINE lines on stderr), for k = 1, 2, 4, 6.
    python tools/tail_probe.py [k ...]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "cuda-raytracer_amd"), os.path.join(REPO, "tools")]
os.environ["RTAMD_TIMELINE"] = "1"
import make_envmap  # noqa: E402
import rtamd  # noqa: E402

make_envmap.ensure_envmap(os.path.join(REPO, "assets", "teapot", "textures", "envmap.pfm"))
ks = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 6]
tag = os.environ.get("PROBE_TAG", "")
scene = rtamd.Scene(os.path.join(rtamd.ASSETS, "teapot.scene"), image=(1920, 1080, 2048, 16))
r = rtamd.Renderer(scene, sort=True)
r.set_event_timing(True)
r.run(0, 2)
for k in ks:
    best = None
    for rep in range(2):
        st = r.run(0, k)
        prof = r.launch_profile()
        if best is None or st["kernel_ms"] < best[0]["kernel_ms"]:
            best = (st, prof)
    st, prof = best
    spans = [round(p[0], 3) for p in prof]
    print(json.dumps({"tag": tag, "passes": k, "kernel_ms": round(st["kernel_ms"], 2), "pass0_trace_ms_by_bounce": spans,
                      "pass0_tail_trace_ms": round(sum(spans[2:]), 3), "process_ms": round(st["process_ms"], 2), "sort_ms": round(st["sort_ms"], 2), "trace_ms": round(st["trace_ms"], 2)}), flush=True)
r.close()
