"""Where the CLI's fixed 'GPU Took' time goes: HIP runtime init vs first render vs warm render."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "cuda-raytracer_amd"))
import rtamd
t = time.perf_counter(); rtamd.lib(); t_lib = time.perf_counter() - t
t = time.perf_counter(); n = rtamd.device_count(); t_init = time.perf_counter() - t
print("load lib %.3f s, hipGetDeviceCount (runtime init) %.3f s, devices %d" % (t_lib, t_init, n))
for spp in (1, 100):
    sc = rtamd.Scene(os.path.join(rtamd.ASSETS, "teapot.scene"), image=(1000, 1000, spp, 10))
    for k in range(3):
        t = time.perf_counter(); fb, st = rtamd.render(sc, sort=True); w = time.perf_counter() - t
        print("spp %d render %d: wall %.3f s, render_ms %.1f, kernel_ms %.1f" % (spp, k, w, st["render_ms"], st["kernel_ms"]))
