"""Render the reference-settings scenes on the GPU and save the raw framebuffers (gpurun_out/)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-raytracer_amd"))
import rtamd as R  # noqa: E402

os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
for scene in sys.argv[1:] or ["cornell", "cornell_plus", "spheres"]:
    sc = R.Scene(os.path.join(R.ASSETS, scene + ".scene"))
    fb, st = R.render(sc, sort=True)
    np.save(os.path.join(REPO, "gpurun_out", "fb_%s.npy" % scene), fb.astype(np.float32))
    print(scene, st["render_ms"])
