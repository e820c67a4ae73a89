"""Parity at the BASELINE configs' full sizes (BASELINE.json configs 1-5), with no oracle code on the
GPU box: the HIP render's raw framebuffer (float32 per-pixel sums, W*H*3) is hashed and compared with
SHA-256 fixtures the CPU oracle produced in the container:

  * tests/golden/bench_pass0.json (make_bench_hashes.py): pass 0 of every workload (cornell 256^2,
    cornell_plus 512^2, spheres 1024^2 no_bvh, teapot 1080p x 16 and lamp 1080p x 32 bounces, both
    sort modes for teapot and lamp);
  * tests/golden/bench_frames.json (make_frame_hashes.py): the whole cornell, cornell_plus and
    spheres frames, the last (remainder) pass of teapot and lamp in both sort modes, and (round 6) the
    whole teapot frames in both sort modes.

Reference loop: raytracing.cu:222-254 (pass rtc / remaining :224-229, process seeds :235, the
reorder :238-247)."""
import hashlib
import json
import os

import numpy as np
import pytest

import rtamd as R

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PASS0 = json.load(open(os.path.join(GOLDEN, "bench_pass0.json")))
FRAMES = json.load(open(os.path.join(GOLDEN, "bench_frames.json")))

CASES = [("pass0 " + k, v["scene"], v["image"], v["use_bvh"], k.endswith("sort=on"), 0, 1, v)
         for k, v in sorted(PASS0.items())] + \
        [(k, v["scene"], v["image"], v["use_bvh"], v["sort"], v["pass_begin"], v["pass_count"], v)
         for k, v in sorted(FRAMES.items())]

_scenes = {}


def scene(name, image, use_bvh):
    key = (name, tuple(image), use_bvh)
    if key not in _scenes:
        _scenes.clear()      # one resident scene at a time (lamp is ~300 k triangles)
        _scenes[key] = R.Scene(os.path.join(R.ASSETS, name), use_bvh=use_bvh, image=tuple(image))
    return _scenes[key]


@pytest.fixture(scope="module")
def gpu():
    if R.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    return 0


@pytest.mark.parametrize("key,name,image,use_bvh,sort,begin,count,gold", CASES, ids=[c[0] for c in CASES])
def test_full_size_bitexact(gpu, key, name, image, use_bvh, sort, begin, count, gold):
    sc = scene(name, image, use_bvh)
    fb, st = R.render(sc, sort=sort, pass_begin=begin, pass_count=count)
    digest = hashlib.sha256(fb.astype("<f4").tobytes()).hexdigest()
    assert st["live_segments"] == gold["live_segments"], key
    if "mean" in gold:
        assert np.allclose(fb.reshape(-1, 3).mean(axis=0), gold["mean"], rtol=1e-5)
    assert digest == gold["sha256"], key
