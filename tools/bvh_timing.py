"""GPU vs host BVH build times (run on the GPU box): RTAMD_TIMING phase breakdown of the GPU
build and the loader's "BVH Took" for both, 3 repeats each after a warm-up.
usage: RTAMD_TIMING=1 python tools/bvh_timing.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-raytracer_amd"))
import rtamd as R  # noqa: E402

R.Scene(os.path.join(R.ASSETS, "cornell.scene"), bvh_device=0)     # HIP start-up
for name in ("teapot", "lamp_available"):
    path = os.path.join(R.ASSETS, name + ".scene")
    for dev in (-1, 0):
        ms = [R.Scene(path, bvh_device=dev).bvh_ms for _ in range(3)]
        print("%-15s %s  BVH ms: %s" % (name, "gpu " if dev >= 0 else "host", " ".join("%.1f" % x for x in ms)),
              flush=True)
