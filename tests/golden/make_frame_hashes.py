"""Generates tests/golden/bench_frames.json: SHA-256 fixtures of the CPU oracle's framebuffers at
the BASELINE configs' full sizes, beyond bench_pass0.json's pass 0:

  * whole frames (every pass, accumulated in pass order) of the configs small enough for the
    oracle to finish in minutes here: cornell 256^2 x 64 spp x 4 (config 1), cornell_plus
    512^2 x 256 spp x 8 (config 2), spheres 1024^2 x 1024 spp x 8 no_bvh (config 3);
  * the LAST (remainder) pass of teapot (config 4, 8 spp, generate seed remaining = 0) and lamp
    (config 5, 16 spp), sort on and off: pass 0 is already pinned, and the last pass is the one
    whose rtc differs (raytracing.cu:224-225);
  * (round 6) the whole teapot frames, sort on and off (lamp's would take ~3.5 h each here).

The GPU tests (tests/test_gpu_baseline_sizes.py) render the same frames / passes through the C ABI
and compare hashes, so no oracle code runs on the GPU box for these sizes.  Reference loop:
raytracing.cu:222-254; seeds raytracing.cu:89, :229, :235.

    python tests/golden/make_frame_hashes.py [key ...]     (run in the container; minutes)
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "tools"), REPO]

import bench  # noqa: E402  (CONFIGS only; importing it runs nothing)
import make_envmap  # noqa: E402
import oracle_lib as O  # noqa: E402

OUT = os.path.join(HERE, "bench_frames.json")

# key: (bench config, sort, what) with what = "frame" (every pass) or "last" (the last pass only)
JOBS = {
    "cornell frame sort=on": ("cornell", True, "frame"),
    "cornell_plus frame sort=on": ("cornell_plus", True, "frame"),
    "spheres frame sort=on": ("spheres", True, "frame"),
    "teapot last sort=on": ("teapot", True, "last"),
    "teapot last sort=off": ("teapot", False, "last"),
    "lamp last sort=on": ("lamp", True, "last"),
    "lamp last sort=off": ("lamp", False, "last"),
    # round 6: the whole teapot frames too (~50 min each here); the lamp frames (~3.5 h each) are not generated
    "teapot frame sort=on": ("teapot", True, "frame"),
    "teapot frame sort=off": ("teapot", False, "frame"),
    "lamp frame sort=on": ("lamp", True, "frame"),
    "lamp frame sort=off": ("lamp", False, "frame"),
}


def main():
    make_envmap.ensure_envmap(os.path.join(REPO, "assets", "teapot", "textures", "envmap.pfm"))
    O.build()
    want = sys.argv[1:] or list(JOBS)
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for k in want:
        name, sort, what = JOBS[k]
        scene_file, W, H, spp, bounces, _, use_bvh = bench.CONFIGS[name]
        P = -(-spp // 20)
        begin, count = (0, P) if what == "frame" else (P - 1, 1)
        t0 = time.time()
        sc = O.OracleScene(os.path.join(REPO, "assets", scene_file), use_bvh=use_bvh, image=(W, H, spp, bounces))
        fb, st = sc.render(sort=sort, pass_begin=begin, pass_count=count)
        out[k] = {"sha256": hashlib.sha256(fb.astype("<f4").tobytes()).hexdigest(),
                  "live_segments": int(st["live_segments"]), "generated_rays": int(st["generated_rays"]),
                  "image": [W, H, spp, bounces], "scene": scene_file, "use_bvh": bool(use_bvh), "sort": sort,
                  "pass_begin": begin, "pass_count": count,
                  "mean": [float(x) for x in fb.reshape(-1, 3).mean(axis=0)]}
        print(k, out[k]["sha256"][:16], "%.1f s" % (time.time() - t0), flush=True)
        json.dump(out, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
