"""Teapot pass 0 rendered alone (one pass context) a few times, for a per-kernel profile of the exclusive
pass:  rocprofv3 --kernel-trace --stats -d gpurun_out/X -o run --output-format csv -- python3 tools/pass_kernels.py
Env: PK_SCENE (teapot.scene), PK_IMAGE (1920,1080,2048,16), PK_RUNS (4), PK_SORT (1)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["RTAMD_INFLIGHT"] = "1"
sys.path[:0] = [os.path.join(REPO, "cuda-raytracer_amd"), os.path.join(REPO, "tools")]
import make_envmap  # noqa: E402
import rtamd  # noqa: E402

make_envmap.ensure_envmap(os.path.join(REPO, "assets", "teapot", "textures", "envmap.pfm"))
scene = rtamd.Scene(os.path.join(rtamd.ASSETS, os.environ.get("PK_SCENE", "teapot.scene")),
                    image=tuple(int(x) for x in os.environ.get("PK_IMAGE", "1920,1080,2048,16").split(",")))
r = rtamd.Renderer(scene, sort=os.environ.get("PK_SORT", "1") != "0")
for k in range(int(os.environ.get("PK_RUNS", "4"))):
    st = r.run(0, 1)
    print("run %d: kernel_ms %.3f" % (k, st["kernel_ms"]), flush=True)
r.close()
