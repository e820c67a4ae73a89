"""One-GPU strong-scaling probe of the in-library multi-GPU path (rt_render with rt_opts.device_count,
csrc/rt_multi.hip): a rank's share of the teapot frame at N = 8 / 4 / 2 is 13 / 26 / 52 passes; render a frame
of that many passes through rt_render(devices=[0]) -- pass sharding over one device, the overlapped RCCL
exchange (or RTAMD_XCHG_OVERLAP=0) -- and report the device loop's ms per pass (render + exchange, without
renderer creation), next to the plain renderer's run of the same passes.
    python tools/share_probe.py [13 26 52]"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys, time
sys.path[:0] = [os.path.join(%(repo)r, "cuda-raytracer_amd"), os.path.join(%(repo)r, "tools")]
import make_envmap, rtamd as R
make_envmap.ensure_envmap(os.path.join(%(repo)r, "assets", "teapot", "textures", "envmap.pfm"))
psc = R.Scene(os.path.join(R.ASSETS, "teapot.scene"), image=(1920, 1080, 20 * %(n)d, 16))
if %(multi)d:
    for k in range(2):
        R.render(psc, sort=True, devices=[0])
else:
    ren = R.Renderer(psc, sort=True)
    ren.set_event_timing(False)
    ren.run(0, %(n)d)
    for k in range(2):
        ren.clear()
        t = time.perf_counter()
        ren.run(0, %(n)d)
        print("plain %%d passes in %%.2f ms" %% (%(n)d, (time.perf_counter() - t) * 1e3), file=sys.stderr)
    ren.close()
"""


def main():
    ns = [int(x) for x in sys.argv[1:]] or [13, 26, 52]
    for n in ns:
        for multi in (0, 1):
            env = dict(os.environ, RTAMD_TIMING="1", GPU_MAX_HW_QUEUES=os.environ.get("GPU_MAX_HW_QUEUES", "24"))
            out = subprocess.run([sys.executable, "-c", CHILD % {"repo": REPO, "n": n, "multi": multi}], env=env,
                                 capture_output=True, text=True, timeout=600)
            if out.returncode:
                print(out.stderr[-3000:])
                sys.exit(1)
            if multi:
                ms = [float(m) for m in re.findall(r"rt_multi device 0: \d+ passes rendered and exchanged in ([\d.]+) ms",
                                                   out.stderr)]
                xs = re.findall(r"exchange not hidden: ([\d.]+) ms", out.stderr)
                gs = re.findall(r"framebuffer to the host ([\d.]+) ms", out.stderr)
                print("%d passes  rt_render(devices=[0]) render+exchange loop %s ms -> best %.3f ms/pass (exchange not "
                      "hidden %s ms; then gather + D2H %s ms)" % (n, ms, min(ms) / n, xs, gs), flush=True)
            else:
                ms = [float(m) for m in re.findall(r"plain \d+ passes in ([\d.]+) ms", out.stderr)]
                print("%d passes  plain renderer run %s ms -> best %.3f ms/pass" % (n, ms, min(ms) / n), flush=True)


if __name__ == "__main__":
    main()
