"""Exclusive trace launches of teapot pass 0 (one pass context, as bench.py exclusive_pass), timed two ways in
one process: the renderer's device wall-clock spans (event timing on) and, under rocprofv3 --kernel-trace, the
profiler's dispatch durations; then the same pass with event timing off (profiler only).
    rocprofv3 --kernel-trace --stats -d DIR -o run --output-format csv -- python3 tools/excl_probe.py"""
import os
import sys

os.environ["RTAMD_INFLIGHT"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "cuda-raytracer_amd"), os.path.join(REPO, "tools")]
import make_envmap  # noqa: E402
import rtamd  # noqa: E402

make_envmap.ensure_envmap(os.path.join(REPO, "assets", "teapot", "textures", "envmap.pfm"))
scene = rtamd.Scene(os.path.join(rtamd.ASSETS, "teapot.scene"), image=(1920, 1080, 2048, 16))
r = rtamd.Renderer(scene, sort=True)
r.set_event_timing(True)
r.run(0, 1)
for k in range(3):
    st = r.run(0, 1)
    print("events on: trace %.3f ms over %d launches = %.4f ms/launch, kernels %.3f ms" % (
        st["trace_ms"], st["trace_launches"], st["trace_ms"] / st["trace_launches"], st["kernel_ms"]), flush=True)
r.set_event_timing(False)
for k in range(3):
    r.run(0, 1)
print("events off: 3 passes (profiler durations only)", flush=True)
r.close()
