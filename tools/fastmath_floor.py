"""How far nvcc --use_fast_math alone moves a rendered image (measurement; test infrastructure only).

The reference's GPU path is built with `nvcc --use_fast_math` (build.sh:2): FMA contraction,
approximate division and square root, __sinf/__cosf (random.cuh:63-75) and FTZ.  It cannot run
here, so its image is never compared directly.  This script renders the same scenes,
seeds and sizes with two builds of the oracle -- the IEEE restatement every parity test uses
(oracle/build/liboracle.so, which the HIP path equals bit for bit) and the fast-math study build
(oracle/build/liboracle_fastmath.so: oracle.cpp under ORC_FASTMATH, compiled with contraction) --
and reports their difference on the normalised linear image (exposure / ray_count) * fb, the
quantity of SURVEY.md §8c's stated tolerance (RMS < 1e-4 per channel).  Next to it, the difference
between two IEEE renders of the same scene with other seeds (the first half of a frame of twice
the passes): the Monte-Carlo noise floor.  Any implementation that differs from the reference only
by fast-math rounding differs from it by about the first figure; no implementation can reach a
per-pixel tolerance below it.

    python tools/fastmath_floor.py [--out docs/history/profiles/r04/fastmath_floor.json]
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))

CASES = [
    # scene, W, H, spp, bounces (20 x 20 block grid: W and H divisible by 20)
    ("cornell_plus.scene", 160, 160, 60, 8),
    ("teapot.scene", 320, 180, 60, 16),
]
FASTMATH_LIB = os.path.join(REPO, "oracle", "build", "liboracle_fastmath.so")
FMA_LIB = os.path.join(REPO, "oracle", "build", "liboracle_fma.so")   # contraction only


def render(scene, w, h, spp, bounces, pass_begin, pass_count, out, threads):
    import oracle_lib as O
    sc = O.OracleScene(os.path.join(O.ASSETS, scene), image=(w, h, spp, bounces))
    fb, st = sc.render(sort=True, pass_begin=pass_begin, pass_count=pass_count, threads=threads)
    np.save(out, fb)
    return st


def run_child(lib, *args):
    env = dict(os.environ)
    if lib:
        env["ORACLE_LIB"] = lib
    subprocess.run([sys.executable, os.path.abspath(__file__), "--render"] + [str(a) for a in args],
                   check=True, env=env, cwd=REPO)


def metrics(a, b, w, h, exposure, ray_count):
    s = exposure / ray_count
    la = (s * a).reshape(h, w, 3).astype(np.float64)
    lb = (s * b).reshape(h, w, 3).astype(np.float64)
    d = la - lb
    bw, bh = w // 20, h // 20
    ba = la.reshape(20, bh, 20, bw, 3).mean(axis=(1, 3))
    bb = lb.reshape(20, bh, 20, bw, 3).mean(axis=(1, 3))
    import oracle_lib as O
    ta = np.zeros(w * h * 3, np.uint8)
    tb = np.zeros(w * h * 3, np.uint8)
    L = O.lib()
    L.orc_tonemap(O.ptr(np.ascontiguousarray(a, np.float32)), w, h, exposure, ray_count, O.ptr(ta))
    L.orc_tonemap(O.ptr(np.ascontiguousarray(b, np.float32)), w, h, exposure, ray_count, O.ptr(tb))
    return {
        "rms": [float(np.sqrt(np.mean(d[..., c] ** 2))) for c in range(3)],
        "max_abs": [float(np.abs(d[..., c]).max()) for c in range(3)],
        "block20_rms": [float(np.sqrt(np.mean((ba - bb)[..., c] ** 2))) for c in range(3)],
        "mean_level": [float(la[..., c].mean()) for c in range(3)],
        "png_bytes_equal": float(np.mean(ta == tb)),
        "png_max_lsb": int(np.abs(ta.astype(int) - tb.astype(int)).max()),
        "pixels_differing": float(np.mean(np.any(d != 0, axis=2))),
    }


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--render":
        a = sys.argv[2:]
        render(a[0], *[int(x) for x in a[1:7]], a[7], int(a[8]))
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r05", "fastmath_floor.json"))
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    import make_envmap
    make_envmap.ensure_envmap(os.path.join(REPO, "assets", "teapot", "textures", "envmap.pfm"))
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    tmp = os.path.join(REPO, "gpurun_out", "fastmath_floor")
    os.makedirs(tmp, exist_ok=True)
    out = {"def": __doc__.strip().split("\n\n")[1].replace("\n", " "),
           "fastmath_build": "oracle/oracle.cpp with -DORC_FASTMATH -ffp-contract=fast -mfma (oracle/Makefile "
                             "FMSTUDY): FMA contraction; a/b as a * float(1/b); sqrt(x) as x * float(1/sqrt(x)) and "
                             "1/sqrt(x) as float(1/sqrt(x)); sin/cos of random_on_sphere with the argument scaled by "
                             "1/(2 pi) in float and the result rounded to 2^-22; FTZ/DAZ",
           "contraction_build": "oracle/oracle.cpp with -ffp-contract=fast -mfma only (nvcc's default -fmad=true)",
           "cases": []}
    import oracle_lib as O
    for scene, w, h, spp, bounces in CASES:
        P = -(-spp // 20)
        f_ieee = os.path.join(tmp, "%s_ieee.npy" % scene)
        f_fm = os.path.join(tmp, "%s_fm.npy" % scene)
        f_seed = os.path.join(tmp, "%s_seed.npy" % scene)
        f_fma = os.path.join(tmp, "%s_fma.npy" % scene)
        run_child(None, scene, w, h, spp, bounces, 0, P, f_ieee, args.threads)
        run_child(FASTMATH_LIB, scene, w, h, spp, bounces, 0, P, f_fm, 1)
        run_child(FMA_LIB, scene, w, h, spp, bounces, 0, P, f_fma, args.threads)
        # other seeds, same estimator: passes 0 .. P-1 of a frame of 2 * spp (seeds follow `remaining`,
        # the samples still to cast, so the LAST P passes of that frame would repeat this one's seeds);
        # spp a multiple of 20 keeps every pass at 20 samples
        run_child(None, scene, w, h, 2 * spp, bounces, 0, P, f_seed, args.threads)
        info = O.OracleScene(os.path.join(O.ASSETS, scene), image=(w, h, spp, bounces)).info
        ieee, fm, seed, fma = np.load(f_ieee), np.load(f_fm), np.load(f_seed), np.load(f_fma)
        case = {"scene": scene, "image": [w, h, spp, bounces], "sort": True,
                "fastmath_vs_ieee": metrics(fm, ieee, w, h, info.exposure, spp),
                "contraction_only_vs_ieee": metrics(fma, ieee, w, h, info.exposure, spp),
                "other_seeds_vs_ieee": metrics(seed, ieee, w, h, info.exposure, spp)}
        out["cases"].append(case)
        print(json.dumps(case), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
