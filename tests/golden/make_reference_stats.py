"""Extract statistical anchors from the reference's own outputs, renders/<scene>.png (run here,
where /root/reference exists; the GPU box only reads the committed JSON).

The PNGs were rendered by the reference GPU path (nvcc --use_fast_math, GTX 1080) at the scene
files' own settings (1000x1000, 1000 spp, 10 bounces); comparison shows they predate the bloom
pass (tests/test_reference_renders.py).  They cannot be matched bit for
bit (fast-math, atomics, FMA contraction), so we keep per-channel means and a 20x20 block-mean
thumbnail per scene, with each block's per-pixel noise variance (for z-scores), and for
cornell_plus the statistics of its emissive, dielectric and mirror regions (primary-hit masks
from the oracle, tests/golden/cornell_plus_regions.npz).  teapot/lamp/glass_teapot used assets missing from the checkout
(.MISSING_LARGE_BLOBS) and are recorded for reference only.

    python tests/golden/make_reference_stats.py [/root/reference]
"""
import json
import os
import sys

import numpy as np
from PIL import Image

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_render_stats.json")


def block_noise_var(img, nb=20):
    """Per 50x50 block and channel: the Monte Carlo noise variance of one pixel, estimated from
    horizontally adjacent pixel pairs inside the block (var(a - b) / 2; image structure adds to
    it, so the estimate errs on the large side)."""
    h, w, _ = img.shape
    bh, bw = h // nb, w // nb
    blk = img.reshape(nb, bh, nb, bw, 3)
    d = np.diff(blk, axis=3)                      # pairs within a block row
    return (d ** 2).mean(axis=(1, 3)) / 2.0


def region_stats(img, mask):
    """Mean per channel, pixel count and per-pixel noise variance (adjacent pairs both inside)."""
    pair = mask[:, 1:] & mask[:, :-1]
    d = (img[:, 1:] - img[:, :-1])[pair]
    return {"pixels": int(mask.sum()), "mean": [round(float(v), 4) for v in img[mask].mean(axis=0)],
            "noise_var": [round(float(v), 4) for v in ((d ** 2).mean(axis=0) / 2.0)]}


def cornell_plus_regions():
    """Pixels whose primary ray (through the pixel centre) first hits the light (emissive), the
    glass sphere (dielectric) or the mirror sphere, from the oracle's closest hit at the scene's
    own camera (scene.cu:62-105): masks for region-restricted comparisons."""
    sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                    os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                 "cuda-raytracer_amd")]
    import oracle_lib as O
    import rtamd as R
    path = os.path.join(R.ASSETS, "cornell_plus.scene")
    v = R.Scene(path).view
    W, H = v.width, v.height
    x = (np.arange(W, dtype=np.float32) + np.float32(0.5)) * np.float32(v.inv_width)
    y = (np.arange(H, dtype=np.float32) + np.float32(0.5)) * np.float32(v.inv_height)
    tl = np.array([v.near_plane_top_left.x, v.near_plane_top_left.y, v.near_plane_top_left.z], np.float32)
    sr = np.array([v.scaled_right.x, v.scaled_right.y, v.scaled_right.z], np.float32)
    su = np.array([v.scaled_up.x, v.scaled_up.y, v.scaled_up.z], np.float32)
    d = tl[None, None, :] + x[None, :, None] * sr[None, None, :] - y[:, None, None] * su[None, None, :]
    d = (d / np.sqrt((d * d).sum(-1, keepdims=True))).astype(np.float32).reshape(-1, 3)
    o = np.broadcast_to(np.array([v.camera_position.x, v.camera_position.y, v.camera_position.z], np.float32), d.shape)
    osc = O.OracleScene(path)
    _, idx, _ = osc.closest_hit(np.concatenate([o, d], axis=1))
    a = osc.arrays()
    mat = a["materials"][a["material_indices"][np.maximum(idx, 0)]]
    hit = idx >= 0
    masks = {"emissive": hit & (mat[:, 8:11].max(axis=1) > 0),
             "dielectric": hit & (mat[:, 11] > 0),
             "mirror": hit & (mat[:, 3] >= 1.0) & (mat[:, 11] == 0)}
    return {k: m.reshape(H, W) for k, m in masks.items()}


def main():
    out = {"source": "reference renders/<scene>.png (1000x1000 RGB8, 1000 spp, 10 bounces, no bloom)",
           "scenes": {}}
    for sc in ("cornell", "cornell_plus", "spheres", "teapot", "lamp", "glass_teapot"):
        img = np.asarray(Image.open(os.path.join(REF, "renders", sc + ".png")).convert("RGB"), dtype=np.float64)
        h, w, _ = img.shape
        thumb = img.reshape(20, h // 20, 20, w // 20, 3).mean(axis=(1, 3))
        out["scenes"][sc] = {
            "width": w, "height": h,
            "channel_mean": [round(float(v), 4) for v in img.reshape(-1, 3).mean(axis=0)],
            "thumb20": np.round(thumb, 3).tolist(),
            "adjacent_pixel_absdiff": round(float(np.abs(np.diff(img, axis=1)).mean()), 4),
            "thumb20_noise_var": np.round(block_noise_var(img), 4).tolist(),
            "assets_available": sc in ("cornell", "cornell_plus", "spheres"),
        }
    masks = cornell_plus_regions()
    img = np.asarray(Image.open(os.path.join(REF, "renders", "cornell_plus.png")).convert("RGB"), dtype=np.float64)
    out["scenes"]["cornell_plus"]["regions"] = {k: region_stats(img, m) for k, m in masks.items()}
    np.savez_compressed(os.path.join(os.path.dirname(OUT), "cornell_plus_regions.npz"),
                        **{k: np.packbits(m.reshape(-1)) for k, m in masks.items()})
    with open(OUT, "w") as f:
        json.dump(out, f)
    print({k: v["channel_mean"] for k, v in out["scenes"].items()})


if __name__ == "__main__":
    main()
