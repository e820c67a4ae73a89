"""GPU binned-SAH build (csrc/bvh_build.hip) against the host build (the reference's recursion,
restated and pinned by tests/test_scene_parity.py): the node array, the triangle order and the
material-index order must be byte-identical, for every shipped scene, the edge scenes, and
random triangle soups full of coordinate ties and -0/+0 pairs (the reference's min/max keeps the
first of equal values, so the sign of a zero bound depends on the order of the triangles)."""
import os

import numpy as np
import pytest

import edge_scenes
import rtamd as R

pytestmark = pytest.mark.gpu

SCENES = ["cornell", "cornell_plus", "spheres", "teapot", "glass_teapot", "lamp_available"]


@pytest.fixture(scope="module")
def gpu():
    if R.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    return 0


def _same(path, use_bvh=True):
    host = R.Scene(path, use_bvh=use_bvh)
    dev = R.Scene(path, use_bvh=use_bvh, bvh_device=0)
    a, b = host.arrays(), dev.arrays()
    for k in ("bvh", "triangles", "material_indices", "camera"):
        assert a[k].tobytes() == b[k].tobytes(), k
    return host, dev


@pytest.mark.parametrize("scene", SCENES)
def test_gpu_build_equals_host_build(gpu, scene):
    _same(os.path.join(R.ASSETS, scene + ".scene"))


def test_gpu_build_no_bvh(gpu):
    _same(os.path.join(R.ASSETS, "cornell.scene"), use_bvh=False)


def test_gpu_build_edge_scenes(gpu, tmp_path):
    for p in edge_scenes.write(str(tmp_path)).values():
        _same(p)


@pytest.mark.parametrize("seed,n", [(1, 3000), (2, 20000), (3, 777), (4, 90000)])   # 90000: chunked huge nodes
def test_gpu_build_random_soup_with_ties(gpu, tmp_path, seed, n):
    rng = np.random.default_rng(seed)
    vals = np.array([-2.0, -1.0, -0.0, 0.0, 0.5, 1.0, 3.0], np.float64)
    lines = [edge_scenes.HEADER]
    for _ in range(n):
        if rng.random() < 0.5:
            v = rng.choice(vals, size=(3, 3))          # ties and signed zeros
        else:
            v = rng.normal(size=(3, 3)) * rng.choice([0.01, 1.0, 100.0])
        lines.append("triangle white " + " ".join(repr(float(x)) for x in v.ravel()) + "\n")
    lines.append("camera position 0 0 -10 forward 0 0 1 up 0 1 0 fov 40\nimage 16 16 1 1 1\n")
    p = tmp_path / ("soup%d.scene" % seed)
    p.write_text("".join(lines))
    host, _ = _same(str(p))
    assert host.view.bvh_node_count > 1


def test_gpu_build_renders_identically(gpu):
    path = os.path.join(R.ASSETS, "teapot.scene")
    img = (64, 36, 20, 8)
    a, _ = R.render(R.Scene(path, image=img), sort=True)
    b, _ = R.render(R.Scene(path, image=img, bvh_device=0), sort=True)
    assert np.array_equal(a, b)


def test_cli_gpu_bvh_png_identical(gpu, tmp_path):
    import subprocess
    args = [R.CLI_PATH, "teapot.scene", "--image", "48", "32", "20", "6", "0.7"]
    a = subprocess.run(args + ["--out", str(tmp_path / "a.png")], cwd=R.ASSETS, capture_output=True, text=True)
    b = subprocess.run(args + ["--gpu-bvh", "--out", str(tmp_path / "b.png")], cwd=R.ASSETS, capture_output=True,
                       text=True)
    assert a.returncode == 0 and b.returncode == 0, a.stdout + b.stdout
    assert "Node count: 81311" in a.stdout and "Node count: 81311" in b.stdout
    assert open(tmp_path / "a.png", "rb").read() == open(tmp_path / "b.png", "rb").read()
