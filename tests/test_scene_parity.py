"""The product's host loader + BVH builder (rt_scene_load) against the oracle's restatement.

The two are independent implementations of scene.cu:491-1036; the arrays they hand to the
render path must be byte-identical (same triangle order after the in-place SAH partition,
same node array, same camera precompute and key bounds)."""
import os

import numpy as np
import pytest

import oracle_lib as O
import rtamd as R

SCENES = [("cornell", True), ("cornell", False), ("cornell_plus", True), ("cornell_plus", False),
          ("spheres", True), ("spheres", False), ("teapot", True), ("glass_teapot", True), ("lamp_available", True)]


@pytest.mark.parametrize("name,bvh", SCENES)
def test_loader_arrays_identical(name, bvh):
    path = os.path.join(R.ASSETS, name + ".scene")
    a = O.OracleScene(path, use_bvh=bvh).arrays()
    b = R.Scene(path, use_bvh=bvh).arrays()
    for k in a:
        assert a[k].tobytes() == b[k].tobytes(), k


@pytest.mark.parametrize("threads", ["1", "2", "3", "16"])
def test_bvh_build_independent_of_threads(threads, monkeypatch):
    """The parallel BVH build (subtrees and chunked scans on threads) emits the serial
    reference build's node array and triangle order for any thread count."""
    monkeypatch.setenv("RT_BVH_THREADS", threads)
    for name in ("teapot", "lamp_available"):
        path = os.path.join(R.ASSETS, name + ".scene")
        a = O.OracleScene(path).arrays()
        b = R.Scene(path).arrays()
        for k in ("bvh", "triangles", "material_indices"):
            assert a[k].tobytes() == b[k].tobytes(), (name, threads, k)


def test_image_override_and_camera():
    path = os.path.join(R.ASSETS, "teapot.scene")
    a = O.OracleScene(path, image=(321, 123, 45, 6), exposure=0.25).arrays()["camera"]
    s = R.Scene(path, image=(321, 123, 45, 6), exposure=0.25)
    assert (s.width, s.height, s.view.ray_count, s.view.bounces) == (321, 123, 45, 6)
    assert s.view.exposure == np.float32(0.25)
    assert a.tobytes() == s.arrays()["camera"].tobytes()


def test_crlf_scene_files(tmp_path):
    """The reference files are CRLF (built on Windows); the loader strips '\\r'."""
    src = open(os.path.join(R.ASSETS, "teapot.scene"), "rb").read()
    crlf = tmp_path / "teapot_crlf.scene"
    crlf.write_bytes(src.replace(b"\n", b"\r\n"))
    a = R.Scene(os.path.join(R.ASSETS, "teapot.scene")).arrays()
    b = R.Scene(str(crlf)).arrays()
    for k in a:
        assert a[k].tobytes() == b[k].tobytes(), k


def test_defaults_without_image_line(tmp_path):
    """scene.cu:571-574: 1920x1080, 1 spp, 3 bounces, exposure 0 when no `image` line."""
    p = tmp_path / "s.scene"
    p.write_text("material m diffuse 0.5 0.5 0.5\nsphere m 0 0 5 1\nsky 1 1 1\n"
                 "camera position 0 0 0 forward 0 0 1 up 0 1 0 fov 40\n")
    s = R.Scene(str(p))
    assert (s.width, s.height, s.view.ray_count, s.view.bounces, s.view.exposure) == (1920, 1080, 1, 3, 0.0)


def test_loader_errors(tmp_path):
    with pytest.raises(R.RtError, match="cannot open scene"):
        R.Scene(str(tmp_path / "missing.scene"))
    p = tmp_path / "bad.scene"
    p.write_text("sphere nomaterial 0 0 0 1\n")
    with pytest.raises(R.RtError, match="unknown material"):
        R.Scene(str(p))
    p.write_text("material m\nply m nowhere.ply\n")
    with pytest.raises(R.RtError, match="cannot open ply"):
        R.Scene(str(p))
