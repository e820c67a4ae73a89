"""Analysis (container only, the CPU oracle; verdict r05 item 6): the distinct scene bytes that the rays one XCD
holds in flight touch at one bounce, under three ways of dealing the live slots to the 8 XCDs -- the product's
contiguous eighths of the sorted slots (= runs of origin octants), round 5's x-th eighth of every bucket (image
bands), and routing by the first depth-d subtree the traversal enters (the top-level treelet).  An XCD's L2 is 4 MB;
a window is the lanes one XCD keeps resident (32 CUs x 4 SIMDs x 8 waves x 64 = 65,536).

    python tools/route_model.py teapot [pass] [bounce] [depth] [window]"""
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
p, bounce, depth, window = (int(x) for x in (a[1:] + ["0", "1", "3", "65536"][len(a[1:]):])[:4])
scene_file, W, H, spp, bounces, sort, use_bvh = bench.CONFIGS[name]
sc = O.OracleScene(os.path.join(REPO, "assets", scene_file), use_bvh=use_bvh, image=(W, H, spp, bounces))
L = O.lib()
L.orc_bounce_working_set.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                     C.c_int]
out = np.zeros(21)
if L.orc_bounce_working_set(sc.h, int(sort), p, bounce, window, depth, 4, out.ctypes.data_as(C.c_void_p), 0):
    raise RuntimeError(L.orc_last_error().decode())
names = ["slot eighths (product)", "eighth of every bucket (round 5)", "first depth-%d subtree" % depth]
res = {"workload": "%s %dx%d, pass %d, bounce %d, window %d rays per XCD" % (scene_file, W, H, p, bounce, window),
       "policies": {}}
for i, n in enumerate(names):
    m, mx, f, share, miss, fetched = out[i * 6:(i + 1) * 6]
    res["policies"][n] = {"distinct_MB_mean": round(m / 2**20, 2), "distinct_MB_max": round(mx / 2**20, 2),
                          "fetched_MB_per_window": round(f / 2**20, 1), "largest_xcd_share": round(share, 3),
                          "l2_miss_GB_bounce": round(miss / 1e9, 3), "fetched_GB_bounce": round(fetched / 1e9, 2)}
res["overflow_stack"] = {"pushes": int(out[18]), "live_rays": int(out[19]), "rays_overflowing": int(out[20]),
                         "bytes_written_and_read_GB": round(out[18] * 8 * 2 / 1e9, 3)}
print(json.dumps(res, indent=1))
