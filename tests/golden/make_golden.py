"""Regenerate the oracle's golden vectors (tests/golden/oracle_kat.json, oracle_fb.npz).

These pin the CPU oracle against regressions and make its edge-case semantics explicit; the
reference itself has no tests or golden vectors to pin against, and its
code may not be run (denied) — see tests/test_oracle_golden.py for the anchors
that do come from the reference (BVH counts, renders/*.png statistics).

    python tests/golden/make_golden.py
"""
import ctypes as C
import hashlib
import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402

F32 = np.float32


def f(x):
    return float(np.float32(x))


def main():
    L = O.lib()
    ptr = O.ptr
    kat = {}
    # --- PCG (random.cuh:13-45)
    kat["pcg"] = {}
    for seed in (0, 1, 12345, 0x85810BEA, 0xFFFFFFFF):
        out = np.zeros(16, np.uint32)
        L.orc_pcg_stream(seed, 16, ptr(out))
        kat["pcg"][str(seed)] = out.tolist()
    r01, r02, rad = (np.zeros(64, F32) for _ in range(3))
    L.orc_random_draws(777, 64, ptr(r01), ptr(r02), ptr(rad))
    kat["draws_777"] = {"random01": r01.tolist(), "random02": r02.tolist(), "random_radians": rad.tolist()}
    ros = np.zeros(64 * 3, F32)
    L.orc_random_on_sphere(4242, 64, ptr(ros))
    kat["random_on_sphere_4242"] = ros.tolist()
    # --- deterministic sin/cos/atan kernels
    xs = np.linspace(0, 2 * math.pi, 257, dtype=np.float64).astype(F32)
    xs = np.concatenate([xs, np.array([0.0, 1e-7, math.pi / 4, math.pi / 2, math.pi, 6.2831855], F32)])
    s, c = np.zeros_like(xs), np.zeros_like(xs)
    L.orc_sincos(ptr(xs), len(xs), ptr(s), ptr(c))
    kat["sincos"] = {"x": xs.tolist(), "sin": s.tolist(), "cos": c.tolist()}
    ats = np.linspace(0, 1, 101).astype(F32)
    kat["atan01"] = {"x": ats.tolist(), "y": [L.orc_atan01(float(v)) for v in ats]}
    # --- seeds (raytracing.cu:89, 148; scene.cu:81)
    idx = [0, 1, 2, 19, 20, 12345, 41471999, 2**31 - 1]
    kat["seeds"] = {"index": idx,
                    "generate": [L.orc_generate_seed(i, s_) for i in idx for s_ in (0, 7, 4076)],
                    "process": [L.orc_process_seed(i, s_) for i in idx for s_ in (0, 15, 81935)],
                    "cpu": [L.orc_cpu_seed(i, s_) for i in idx for s_ in (0, 7, 4076)]}
    # --- morton / key buckets (scene.cu:44-60)
    xs = [0.0, -0.0, 0.01, 0.03125, 0.05, 0.5, 0.99, 1.0, 1.5, 2.3, -1.0, float("nan"), float("inf"),
          float("-inf"), 3000.0, 1e9]
    kat["morton"] = [[x, L.orc_morton(x, 0.0, 0.0), L.orc_morton(0.0, x, 0.0), L.orc_morton(0.0, 0.0, x)] for x in xs]
    keys = [0, 0x41, 0x82, 0x104, 0x1C7, 0x410000, 0x1C701C7, 0xFFFFFFFF]
    kat["key_bucket"] = [[k, L.orc_key_bucket(k)] for k in keys]
    # --- slab test (scene.cu:109-132), including 0*inf NaNs
    cases = []
    for (bmin, bmax, o, d, tmax) in [
        ((0, 0, 0), (1, 1, 1), (-1, 0.5, 0.5), (1, 0, 0), 1e30),
        ((0, 0, 0), (1, 1, 1), (-1, 0.5, 0.5), (-1, 0, 0), 1e30),
        ((0, 0, 0), (1, 1, 1), (0, 0.5, 0.5), (0, 1, 0), 1e30),      # origin on the min x plane, d.x = 0
        ((0, 0, 0), (1, 1, 1), (0.5, 0.5, 0.5), (0.3, 0.4, 0.5), 0.1),
        ((0, 0, 0), (0, 1, 1), (-2, 0.5, 0.5), (1, 0, 0), 1e30),      # flat box
        ((-1e30, -1e30, -1e30), (1e30, 1e30, 1e30), (0, 0, 0), (0.6, 0.8, 0.0), 5.0)]:
        a, b, oo, dd = (np.array(v, F32) for v in (bmin, bmax, o, d))
        tmin = np.zeros(1, F32)
        hit = L.orc_ray_aabb(ptr(a), ptr(b), ptr(oo), ptr(dd), tmax, ptr(tmin))
        cases.append({"bmin": bmin, "bmax": bmax, "o": o, "d": d, "tmax": tmax, "hit": hit, "tmin": float(tmin[0])})
    kat["slab"] = cases
    # --- Möller–Trumbore (scene.cu:166-191): the 0.005 threshold is a double compare
    tri = np.array([0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1], F32)       # p1, e1, e2, normal
    mt = []
    for z0 in (np.float32(-0.005), np.float32(-float.fromhex("0x1.47ae16p-8")), np.float32(-1.0), np.float32(-0.004)):
        o = np.array([0.25, 0.25, z0], F32)
        d = np.array([0, 0, 1], F32)
        t = np.zeros(1, F32)
        hit = L.orc_ray_triangle(ptr(tri), ptr(o), ptr(d), 1e30, ptr(t))
        mt.append({"o": o.tolist(), "hit": hit, "t": float(t[0]) if hit else None})
    o = np.array([0.25, 0.25, -1], F32)
    d = np.array([1, 0, 0], F32)                                   # parallel: a == 0
    t = np.zeros(1, F32)
    mt.append({"o": o.tolist(), "d": d.tolist(), "hit": L.orc_ray_triangle(ptr(tri), ptr(o), ptr(d), 1e30, ptr(t))})
    kat["moller_trumbore"] = mt
    # --- sphere (scene.cu:340-371)
    sph = np.array([0, 0, 5, 1], F32)
    sp = []
    for oz in (0.0, 4.0, 4.0 + 2 ** -9, 7.0):
        o = np.array([0, 0, oz], F32)
        d = np.array([0, 0, 1], F32)
        t = np.zeros(1, F32)
        hit = L.orc_ray_sphere(ptr(sph), ptr(o), ptr(d), 1e30, ptr(t))
        sp.append({"oz": oz, "hit": hit, "t": float(t[0]) if hit else None})
    kat["sphere"] = sp
    # --- environment projection (scene.cu:284-318, 380-391)
    dirs = [(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1), (0.6, 0.8, 0), (0.3, -0.4, -0.866),
            (-0.5, 0.5, 0.70710678), (0.1, 0.9, -0.42)]
    env = []
    for dv in dirs:
        dd = np.array(dv, F32)
        uv = np.zeros(2, F32)
        L.orc_env_project(ptr(dd), ptr(uv))
        env.append({"d": list(dv), "uv": uv.tolist(), "texel_1024": L.orc_env_texel(ptr(dd), 1024, 1024),
                    "texel_1": L.orc_env_texel(ptr(dd), 1, 1)})
    kat["env"] = env
    # --- scenes: counts and array hashes (scene.cu:569-1036)
    scenes = {}
    for name, bvh in (("cornell", True), ("cornell", False), ("cornell_plus", True), ("spheres", True),
                      ("teapot", True), ("lamp_available", True)):
        sc = O.OracleScene(os.path.join(O.ASSETS, name + ".scene"), use_bvh=bvh)
        a = sc.arrays()
        h = hashlib.sha256()
        for k in ("spheres", "triangles", "material_indices", "materials", "bvh", "camera"):
            h.update(a[k].tobytes())
        scenes["%s%s" % (name, "" if bvh else "_no_bvh")] = {
            "triangles": sc.info.triangle_count, "spheres": sc.info.sphere_count,
            "nodes": sc.info.bvh_node_count, "sha256": h.hexdigest()}
    kat["scenes"] = scenes
    with open(os.path.join(HERE, "oracle_kat.json"), "w") as fh:
        json.dump(kat, fh, indent=0)
    # --- small framebuffers + per-bounce bucket histograms
    fbs = {}
    for name, img, sort in (("cornell", (32, 32, 24, 4), True), ("cornell", (32, 32, 24, 4), False),
                            ("cornell_plus", (32, 32, 20, 8), True), ("spheres", (32, 24, 20, 8), True),
                            ("teapot", (48, 27, 20, 16), True)):
        sc = O.OracleScene(os.path.join(O.ASSETS, name + ".scene"), image=img)
        fb, st, hist = sc.render(sort=sort, hist=True)
        key = "%s_%dx%dx%dx%d_%s" % (name, *img, "sort" if sort else "nosort")
        fbs[key + "_fb"] = fb
        fbs[key + "_hist"] = hist
        fbs[key + "_stats"] = np.array([st[k] for k in ("live_segments", "nodes_popped", "internal_visits",
                                                        "triangle_tests", "misses")], np.uint64)
    np.savez_compressed(os.path.join(HERE, "oracle_fb.npz"), **fbs)
    print("wrote oracle_kat.json and oracle_fb.npz")


if __name__ == "__main__":
    main()
