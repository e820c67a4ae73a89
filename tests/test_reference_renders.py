"""Statistical anchor against the reference's own outputs (renders/<scene>.png).

Renders cornell / cornell_plus / spheres at the scene files' own settings (1000x1000, 1000 spp,
10 bounces, sort on) through the product path (rt_render -> rt_tonemap) and compares per-channel
means and 20x20 block means of the 8-bit image with the reference's PNGs.

Finding (round 1): the shipped PNGs were rendered WITHOUT the bloom pass that raytracing.cu:356-393
now applies: without bloom our means match to 0.006-0.02 levels (block RMS 0.07-0.26), with bloom
they are 0.16-1.1 levels brighter everywhere.  So the bloom stage is checked bit-exactly against
the oracle elsewhere and left out of this statistical comparison.  Bit equality with the PNGs is
impossible (nvcc --use_fast_math, FMA contraction, unordered float atomics, independent Monte
Carlo noise), so the block comparison is a z-score against the two estimates' own noise (per-block
pixel noise variance from adjacent pixel pairs), and cornell_plus is also compared on its
emissive, dielectric and mirror regions alone.  teapot/lamp/glass_teapot are not
compared: their assets are missing upstream."""
import json
import os

import numpy as np
import pytest

import rtamd as R

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
STATS = json.load(open(os.path.join(HERE, "golden", "reference_render_stats.json")))["scenes"]
SYSTEMATIC = 0.05   # 8-bit levels: the fast-math / tone-map rounding floor of a block-mean difference


@pytest.mark.parametrize("scene", ["cornell", "cornell_plus", "spheres"])
def test_matches_reference_render_statistics(scene):
    if R.device_count() < 1:
        pytest.fail("no HIP device")
    sc = R.Scene(os.path.join(R.ASSETS, scene + ".scene"))
    v = sc.view
    assert (v.width, v.height, v.ray_count, v.bounces) == (1000, 1000, 1000, 10)
    fb, st = R.render(sc, sort=True)
    img = R.tonemap(fb, v.width, v.height, v.exposure, v.ray_count).reshape(1000, 1000, 3).astype(np.float64)
    ref = STATS[scene]
    mean = img.reshape(-1, 3).mean(axis=0)
    thumb = img.reshape(20, 50, 20, 50, 3).mean(axis=(1, 3))
    dmean = np.abs(mean - np.array(ref["channel_mean"]))
    dthumb = np.abs(thumb - np.array(ref["thumb20"]))
    print(scene, "mean", mean.round(3), "ref", ref["channel_mean"], "max |dmean| %.3f" % dmean.max(),
          "thumb rms %.3f max %.3f" % (np.sqrt((dthumb ** 2).mean()), dthumb.max()),
          "render %.1f ms" % st["render_ms"])
    assert dmean.max() < 0.1
    # Noise-aware block comparison: each 50x50 block mean of two independent 1000-spp estimates
    # differs by Monte Carlo noise of variance (v_ours + v_ref) / 2500, v = that block's per-pixel
    # noise variance from adjacent-pixel pairs (tests/golden/make_reference_stats.py)
    v_ref = np.array(ref["thumb20_noise_var"])
    v_our = block_noise_var(img)
    # + a systematic floor of 0.05 levels: in near-noiseless blocks (spheres' sky: per-pixel variance
    # 0.3) the estimates differ by ~0.1 level, the size of one-LSB tone-map rounding flips between
    # nvcc --use_fast_math and IEEE arithmetic on a fraction of the pixels
    z = (thumb - np.array(ref["thumb20"])) / np.sqrt((v_ref + v_our) / 2500.0 + SYSTEMATIC ** 2)
    print(scene, "block z: rms %.2f max %.2f, |z|>3: %d of %d" % (np.sqrt((z ** 2).mean()), np.abs(z).max(),
                                                                (np.abs(z) > 3).sum(), z.size))
    for k in np.argsort(-np.abs(z).reshape(-1))[:6]:
        by, bx, ch = np.unravel_index(k, z.shape)
        print("  block (%2d,%2d) ch %d: ours %.2f ref %.2f z %.2f (v %.1f / %.1f)" % (
            by, bx, ch, thumb[by, bx, ch], ref["thumb20"][by][bx][ch], z[by, bx, ch], v_our[by, bx, ch], v_ref[by, bx, ch]))
    assert np.sqrt((z ** 2).mean()) < 1.6
    assert np.abs(z).max() < 6.0
    assert (np.abs(z) > 3).sum() <= 0.02 * z.size
    # image noise (adjacent-pixel differences) is that of the reference's 1000-spp estimate
    noise = np.abs(np.diff(img, axis=1)).mean()
    assert abs(noise - ref["adjacent_pixel_absdiff"]) < 0.05 * ref["adjacent_pixel_absdiff"]
    if scene == "cornell_plus":
        check_regions(img, ref["regions"])


def block_noise_var(img, nb=20):
    h, w, _ = img.shape
    d = np.diff(img.reshape(nb, h // nb, nb, w // nb, 3), axis=3)
    return (d ** 2).mean(axis=(1, 3)) / 2.0


def check_regions(img, regions):
    """cornell_plus's emissive (light quad), dielectric (glass sphere) and mirror regions: pixels
    whose primary ray first hits them (oracle closest hit, tests/golden/cornell_plus_regions.npz).
    The glass sphere exercises the dielectric branch (Schlick, TIR, refraction, scene.cu:443-476)
    and the env-lit caustic paths behind it; the light is pure emission (scene.cu:417)."""
    packed = np.load(os.path.join(HERE, "golden", "cornell_plus_regions.npz"))
    for name, rs in regions.items():
        m = np.unpackbits(packed[name])[:img.shape[0] * img.shape[1]].reshape(img.shape[:2]).astype(bool)
        assert m.sum() == rs["pixels"]
        mean = img[m].mean(axis=0)
        pair = m[:, 1:] & m[:, :-1]
        d = (img[:, 1:] - img[:, :-1])[pair]
        v_our = (d ** 2).mean(axis=0) / 2.0
        delta = mean - np.array(rs["mean"])
        z = delta / np.sqrt((v_our + np.array(rs["noise_var"])) / rs["pixels"] + 1e-12)
        print("  region %-10s %6d px  mean %s ref %s  z %s" % (name, rs["pixels"], mean.round(3), rs["mean"], z.round(2)))
        if name == "emissive":
            # pure emission: every sample of a covered pixel is exp-mapped 30 -> byte 251; only the
            # light's edge pixels vary
            assert np.abs(delta).max() < 0.05
        else:
            assert np.abs(z).max() < 5.0, name
