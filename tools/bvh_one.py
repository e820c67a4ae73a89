import os, sys
sys.path.insert(0, "cuda-raytracer_amd")
import rtamd as R
R.Scene(os.path.join(R.ASSETS, "lamp_available.scene"), bvh_device=0)
