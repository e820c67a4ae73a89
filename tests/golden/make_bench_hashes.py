"""Generates tests/golden/bench_pass0.json: the SHA-256 of the CPU oracle's pass-0 framebuffer
(raw per-pixel sums, float32, W*H*3) for every bench.py workload at its full BASELINE size, so
bench.py can report `bit_exact_vs_oracle` by hashing its own pass 0 with no oracle code on the
GPU box.  Pass 0 casts 20 rays/pixel with generate seed `remaining` = spp - 20
(raytracing.cu:222-229) and runs every bounce; with the reorder on its process seeds follow the
post-sort slots (raytracing.cu:89, :238-247), so one pass exercises the whole hot path.

    python tests/golden/make_bench_hashes.py [scene ...]     (run in the container; minutes)
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

OUT = os.path.join(HERE, "bench_pass0.json")


def key(scene, sort):
    return "%s sort=%s" % (scene, "on" if sort else "off")


def main():
    make_envmap.ensure_envmap(os.path.join(REPO, "assets", "teapot", "textures", "envmap.pfm"))
    O.build()
    want = sys.argv[1:] or list(bench.CONFIGS)
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in want:
        scene_file, W, H, spp, bounces, sort, use_bvh = bench.CONFIGS[name]
        for s in ((True, False) if name in ("teapot", "lamp") else (sort,)):
            t0 = time.time()
            sc = O.OracleScene(os.path.join(REPO, "assets", scene_file), use_bvh=use_bvh, image=(W, H, spp, bounces))
            fb, st = sc.render(sort=s, pass_begin=0, pass_count=1)
            out[key(name, s)] = {"sha256": hashlib.sha256(fb.astype("<f4").tobytes()).hexdigest(),
                                 "live_segments": int(st["live_segments"]),
                                 "image": [W, H, spp, bounces], "scene": scene_file, "use_bvh": bool(use_bvh)}
            print(key(name, s), out[key(name, s)]["sha256"][:16], "%.1f s" % (time.time() - t0), flush=True)
            json.dump(out, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
