"""Statistical anchor against the reference's own outputs (renders/<scene>.png).

Renders cornell / cornell_plus / spheres at the scene files' own settings (1000x1000, 1000 spp,
10 bounces, sort on) through the product path (rt_render -> rt_tonemap) and compares per-channel
means and 20x20 block means of the 8-bit image with the reference's PNGs.

Finding (round 1): the shipped PNGs were rendered WITHOUT the bloom pass that raytracing.cu:356-393
now applies: without bloom our means match to 0.006-0.02 levels (block RMS 0.07-0.26), with bloom
they are 0.16-1.1 levels brighter everywhere.  So the bloom stage is checked bit-exactly against
the oracle elsewhere and left out of this statistical comparison.  Bit equality with the PNGs is
impossible (nvcc --use_fast_math, FMA contraction, unordered float atomics, independent Monte
Carlo noise); the bounds are ~4x the differences measured.  teapot/lamp/glass_teapot are not
compared: their assets are missing upstream."""
import json
import os

import numpy as np
import pytest

import rtamd as R

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
STATS = json.load(open(os.path.join(HERE, "golden", "reference_render_stats.json")))["scenes"]


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
    assert np.sqrt((dthumb ** 2).mean()) < 1.0
    assert dthumb.max() < 6.0
    # image noise (adjacent-pixel differences) is that of the reference's 1000-spp estimate
    noise = np.abs(np.diff(img, axis=1)).mean()
    assert abs(noise - ref["adjacent_pixel_absdiff"]) < 0.05 * ref["adjacent_pixel_absdiff"]
