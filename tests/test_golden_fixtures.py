"""The full-size SHA-256 fixtures (tests/golden/bench_pass0.json, bench_frames.json) describe exactly the
BASELINE workloads bench.py runs (its CONFIGS), so the GPU tests that hash against them
(tests/test_gpu_baseline_sizes.py) cover configs 1-5 at their full sizes.  CPU only."""
import json
import os

import bench

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_pass0_fixtures_match_bench_configs():
    d = json.load(open(os.path.join(GOLDEN, "bench_pass0.json")))
    for name, (scene, W, H, spp, bounces, _sort, use_bvh) in bench.CONFIGS.items():
        keys = [k for k in d if k.split()[0] == name]
        assert keys, name
        for k in keys:
            assert d[k]["image"] == [W, H, spp, bounces] and d[k]["scene"] == scene and d[k]["use_bvh"] == use_bvh
            assert len(d[k]["sha256"]) == 64


def test_frame_fixtures_cover_configs_2_to_5():
    d = json.load(open(os.path.join(GOLDEN, "bench_frames.json")))
    want = {"cornell frame sort=on", "cornell_plus frame sort=on", "spheres frame sort=on",
            "teapot last sort=on", "teapot last sort=off", "lamp last sort=on", "lamp last sort=off"}
    assert want <= set(d)
    for k, v in d.items():
        name = k.split()[0]
        scene, W, H, spp, bounces, _sort, use_bvh = bench.CONFIGS[name]
        P = -(-spp // 20)
        assert v["image"] == [W, H, spp, bounces] and v["scene"] == scene and v["use_bvh"] == use_bvh
        if " frame " in k:
            assert (v["pass_begin"], v["pass_count"]) == (0, P)
        else:
            assert (v["pass_begin"], v["pass_count"]) == (P - 1, 1)
        assert v["sort"] == k.endswith("sort=on")
        assert v["live_segments"] > 0 and len(v["sha256"]) == 64
