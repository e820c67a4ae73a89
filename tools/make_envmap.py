"""Deterministic stand-in for the missing `teapot/textures/envmap.pfm` (.MISSING_LARGE_BLOBS:3).

The reference's teapot/lamp/glass_teapot scenes load a pbrt-v4 equal-area square environment map
that is absent from the reference checkout.  This script writes a procedural square HDR map
(gradient sky + a bright sun disc with a soft glow) in the raw PFM layout load_pfm reads
(scene.cu:548-567: 3 header lines, then W*H float RGB, no row flip).  Only IEEE-exact float32
operations (+ - * / sqrt) are used, so the bytes are identical on every machine.

    python tools/make_envmap.py [out_path] [size]
"""
import hashlib
import os
import sys

import numpy as np


def make_envmap(size: int = 1024) -> np.ndarray:
    f = np.float32
    idx = (np.arange(size, dtype=f) + f(0.5)) / f(size)
    v, u = np.meshgrid(idx, idx, indexing="ij")          # row = v, column = u
    top = np.array([0.30, 0.50, 1.00], dtype=f)
    horizon = np.array([1.00, 0.90, 0.75], dtype=f)
    t = np.sqrt(v)[..., None]
    sky = top[None, None, :] * (f(1) - t) + horizon[None, None, :] * t
    du = u - f(0.70)
    dv = v - f(0.30)
    d2 = du * du + dv * dv
    glow = f(2.0) / (f(1.0) + d2 * f(400.0))
    disc = (d2 < f(0.03 * 0.03)).astype(f) * f(60.0)
    sun = np.array([1.00, 0.95, 0.80], dtype=f)
    img = sky + (glow + disc)[..., None] * sun[None, None, :]
    return img.astype(f)


def write_pfm(path: str, img: np.ndarray) -> str:
    h, w, _ = img.shape
    data = b"PF\n%d %d\n-1.0\n" % (w, h) + np.ascontiguousarray(img, dtype="<f4").tobytes()
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "wb") as fh:
        fh.write(data)
    return hashlib.sha256(data).hexdigest()


def ensure_envmap(path: str, size: int = 1024) -> str:
    if not os.path.exists(path):
        return write_pfm(path, make_envmap(size))
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(__file__), "..", "assets", "teapot", "textures", "envmap.pfm")
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    print(write_pfm(out, make_envmap(size)))
