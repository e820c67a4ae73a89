"""Per-bounce profile of one full-size pass from the CPU oracle (container only; TEST/ANALYSIS
infrastructure): the longest ray's trace steps (internal visits + triangle tests; one HIP trace
step each) and the live rays per bounce -- the floor of a latency-bound tail bounce is that
longest ray's chain of dependent steps.

    python tools/oracle_bounce_profile.py teapot [pass ...] > /tmp/oracle_bounce_profile_teapot.json"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "tools"), REPO]
import bench  # noqa: E402  (CONFIGS only)
import oracle_lib as O  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "teapot"
scene_file, W, H, spp, bounces, sort, use_bvh = bench.CONFIGS[name]
P = -(-spp // 20)
passes = [int(x) for x in sys.argv[2:]] or [0, P - 1]
sc = O.OracleScene(os.path.join(REPO, "assets", scene_file), use_bvh=use_bvh, image=(W, H, spp, bounces))
out = {"workload": "%s %dx%d %dspp %d bounces sort=%s" % (scene_file, W, H, spp, bounces, "on" if sort else "off"),
       "def": "per bounce: max_steps = the longest ray's internal visits + triangle tests (HIP trace steps), "
              "live = live rays (oracle, GPU semantics, tools/oracle_bounce_profile.py)", "passes": {}}
for p in passes:
    steps, live = sc.bounce_profile(sort, p)
    out["passes"][str(p)] = {"max_steps": [int(x) for x in steps], "live": [int(x) for x in live]}
print(json.dumps(out, indent=1))
