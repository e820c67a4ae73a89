"""The product's `cpu` path, tone map, PNG writer and CLI behaviour (all host-side, no GPU).

rt_cpu_render (raytracing.cu:122-163) shares its per-ray arithmetic with the HIP kernels
(rt_device.h, compiled for the host); comparing it bit for bit with the oracle's CPU-path
restatement checks that shared arithmetic on the host, independently of the GPU."""
import os
import subprocess
import zlib

import numpy as np
import pytest

import oracle_lib as O
import rtamd as R


@pytest.mark.parametrize("scene,image", [("cornell", (40, 40, 24, 4)), ("cornell_plus", (32, 32, 20, 6)),
                                         ("spheres", (32, 24, 20, 6)), ("teapot", (48, 27, 20, 8))])
def test_cpu_path_bitexact(scene, image):
    path = os.path.join(R.ASSETS, scene + ".scene")
    ofb, _ = O.OracleScene(path, image=image).render_cpu_path()
    pfb, _ = R.cpu_render(R.Scene(path, image=image), threads=4)
    assert np.array_equal(ofb, pfb)


def test_cpu_path_config1_full_size():
    """BASELINE.json configs[0]: cornell.scene 256x256, 64 spp, 4 bounces through the product's
    `cpu` path (rt_cpu_render, the drop-in for cpu_raytrace, raytracing.cu:122-163: four passes
    of 20/20/20/4 rays per pixel, bounce-invariant seed :148), bit-exact against the oracle's
    restatement at its full size (no GPU needed)."""
    path = os.path.join(R.ASSETS, "cornell.scene")
    image = (256, 256, 64, 4)
    ofb, _ = O.OracleScene(path, image=image).render_cpu_path(threads=8)
    pfb, secs = R.cpu_render(R.Scene(path, image=image), threads=8)
    assert np.array_equal(ofb, pfb)
    assert np.isfinite(pfb).all() and pfb.mean() > 0
    assert secs > 0


def test_tonemap_matches_oracle():
    rng = np.random.default_rng(0)
    fb = (rng.random(300 * 3) * 50).astype(np.float32)
    fb[:3] = [0, 1e30, np.nan]
    assert np.array_equal(R.tonemap(fb, 30, 10, 0.7, 20), O.tonemap(fb, 30, 10, 0.7, 20))


def _decode_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", None, None
    while pos < len(data):
        n = int.from_bytes(data[pos:pos + 4], "big")
        kind = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        crc = int.from_bytes(data[pos + 8 + n:pos + 12 + n], "big")
        assert crc == zlib.crc32(kind + body) & 0xFFFFFFFF
        if kind == b"IHDR":
            w, h = int.from_bytes(body[:4], "big"), int.from_bytes(body[4:8], "big")
            assert body[8:10] == b"\x08\x02"
        elif kind == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = np.frombuffer(raw, np.uint8).reshape(h, w * 3 + 1)
    assert (rows[:, 0] == 0).all()
    return rows[:, 1:].reshape(h, w, 3)


def test_png_roundtrip(tmp_path):
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (70, 130, 3), dtype=np.uint8)      # > 65535 B: several stored blocks
    p = str(tmp_path / "x.png")
    R.write_png(p, img, 130, 70)
    assert np.array_equal(_decode_png(p), img)


def _cli(args, cwd):
    return subprocess.run([R.CLI_PATH] + args, cwd=cwd, capture_output=True, text=True, timeout=300)


def test_cli_usage_and_hardware_errors(tmp_path):
    r = _cli([], tmp_path)
    assert r.returncode == 1 and r.stdout.startswith("Usage: ")
    r = _cli(["x.scene", "no_gpu"], tmp_path)
    assert r.returncode == 2 and r.stdout.strip() == "No raytracing hardware specified"


def test_cli_cpu_only_renders_png(tmp_path):
    """`raytracing <scene> cpu no_gpu` (assets relative to the CWD, like the reference)."""
    r = _cli([os.path.join(R.ASSETS, "cornell_plus.scene"), "cpu", "no_gpu", "--image", "32", "24", "20", "4", "1",
              "unknown_word_is_ignored"], R.ASSETS)
    out = os.path.join(R.ASSETS, "raytracing.png")
    try:
        assert r.returncode == 0, r.stdout + r.stderr
        assert "Triangle count: 32" in r.stdout and "Node count: 21" in r.stdout and "CPU Took" in r.stdout
        img = _decode_png(out)
        sc = O.OracleScene(os.path.join(R.ASSETS, "cornell_plus.scene"), image=(32, 24, 20, 4))
        fb, _ = sc.render_cpu_path()
        want = O.tonemap(fb, 32, 24, 1.0, 20).reshape(24, 32, 3)
        assert np.array_equal(img, want)
    finally:
        if os.path.exists(out):
            os.remove(out)
