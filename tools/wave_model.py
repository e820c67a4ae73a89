"""Analysis (container only, the CPU oracle): would a finer trace order make the trace kernel's waves more coherent?
Replays every live ray's fetch sequence of one bounce through a model 64-lane wave with the kernel's refill rule, in
slot order and in slot order re-sorted within tiles by a finer (origin, direction) key (oracle.cpp
orc_bounce_wave_model).  Slots, seeds and results would not change -- only which rays share a wave.

    python tools/wave_model.py teapot [pass] [bounce] [tile] [obits] [dbits] [refill]"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "tools"), REPO]
import bench  # noqa: E402  (CONFIGS only)
import oracle_lib as O  # noqa: E402

a = sys.argv[1:]
name = a[0] if a else "teapot"
p, bounce, tile, ob, db, refill = (int(x) for x in (a[1:] + ["0", "1", "4096", "4", "2", "24"][len(a[1:]):])[:6])
scene_file, W, H, spp, bounces, sort, use_bvh = bench.CONFIGS[name]
sc = O.OracleScene(os.path.join(REPO, "assets", scene_file), use_bvh=use_bvh, image=(W, H, spp, bounces))
L = O.lib()
L.orc_bounce_wave_model.argtypes = [C.c_void_p] + [C.c_int] * 7 + [C.c_void_p, C.c_int]
out = np.zeros(12)
if L.orc_bounce_wave_model(sc.h, int(sort), p, bounce, tile, ob, db, refill, out.ctypes.data_as(C.c_void_p), 0):
    raise RuntimeError(L.orc_last_error().decode())
res = {"workload": "%s %dx%d pass %d bounce %d; tile %d, origin %d / direction %d bits per axis, refill at %d idle"
       % (scene_file, W, H, p, bounce, tile, ob, db, refill), "orders": {}}
for i, n in enumerate(["slot order", "fine key within tiles"]):
    it, itn, itt, lanes, lines, longest = out[i * 6:(i + 1) * 6]
    res["orders"][n] = {"iterations": int(it), "node_body_iters": int(itn), "tri_body_iters": int(itt),
                        "lane_util_per_body": round(lanes / (64 * (itn + itt)), 4), "lines_per_iter": round(lines / it, 2),
                        "line_requests": int(lines), "longest_ray_steps": int(longest)}
print(json.dumps(res, indent=1))
