"""Analysis (container only, the CPU oracle): per bounce of one full-size pass, the longest ray's chain of
dependent record fetches -- what bounds a latency-bound tail bounce -- and the fetches summed over the live rays,
under the trace-kernel models of oracle.cpp Counters::max_chain:
  cur   one fetch per internal step (root free) and per triangle (the round-5 kernel)
  tl1   two-level records: a descent fetches its node's record and the children's pair together (a fetch serves
        two levels), a stack pop one level; two triangles per fetch
  tl2   as tl1 with the pair index kept on the stack (pops serve two levels too)
  tl1t1 as tl1, one triangle per fetch

    python tools/chain_models.py teapot [pass ...]"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "tools"), REPO]
import bench  # noqa: E402  (CONFIGS only)
import oracle_lib as O  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "teapot"
scene_file, W, H, spp, bounces, sort, use_bvh = bench.CONFIGS[name]
P = -(-spp // 20)
passes = [int(x) for x in sys.argv[2:]] or [0]
sc = O.OracleScene(os.path.join(REPO, "assets", scene_file), use_bvh=use_bvh, image=(W, H, spp, bounces))
L = O.lib()
L.orc_pass_chain_profile.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int]
names = ["cur", "tl1", "tl2", "tl1t1"]
out = {"workload": "%s %dx%d %dspp %d bounces" % (scene_file, W, H, spp, bounces), "models": __doc__.split("\n")[4:12],
       "passes": {}}
for p in passes:
    a = np.zeros((bounces, 8), np.uint64)
    if L.orc_pass_chain_profile(sc.h, int(sort), p, a.ctypes.data_as(C.c_void_p), 0):
        raise RuntimeError(L.orc_last_error().decode())
    rows = []
    for b in range(bounces):
        rows.append({"bounce": b, "max": dict(zip(names, map(int, a[b, :4]))), "sum": dict(zip(names, map(int, a[b, 4:])))})
    tot_max = {n: sum(r["max"][n] for r in rows) for n in names}
    tail_max = {n: sum(r["max"][n] for r in rows if r["bounce"] >= 2) for n in names}
    tot_sum = {n: sum(r["sum"][n] for r in rows) for n in names}
    out["passes"][str(p)] = {"bounces": rows, "max_summed_over_bounces": tot_max, "tail_max_summed": tail_max,
                             "fetches_summed": tot_sum}
print(json.dumps(out, indent=1))
