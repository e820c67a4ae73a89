"""CPU side of the synthetic edge-case scenes (tests/edge_scenes.py): the product loader and the
oracle build the same arrays, and the BVHs have the shapes the GPU tests rely on (a leaf above
the 63 triangles a leaf ref holds inline; a 30-level chain that overflows the trace kernel's
8-entry LDS stack)."""
import numpy as np
import pytest

import edge_scenes
import oracle_lib as O
import rtamd as R


@pytest.fixture(scope="module")
def paths(tmp_path_factory):
    return edge_scenes.write(str(tmp_path_factory.mktemp("edge")))


def _bvh_shape(arrays):
    bvh = arrays["bvh"].view(np.int32).reshape(-1, 8)
    c1, c2 = bvh[:, 6], bvh[:, 7]                 # scene.cuh:82-100: leaf when child2 <= child1
    leaf = c2 <= c1
    depth, deepest, todo = {0: 1}, 1, [0]
    while todo:
        i = todo.pop()
        if not leaf[i]:
            for c in (c1[i], c2[i]):
                depth[c] = depth[i] + 1
                deepest = max(deepest, depth[c])
                todo.append(c)
    return int((c1 - c2)[leaf].max()), deepest


@pytest.mark.parametrize("name", ["big_leaf", "deep"])
def test_loader_matches_oracle(paths, name):
    got, want = R.Scene(paths[name]).arrays(), O.OracleScene(paths[name]).arrays()
    for k in ("spheres", "triangles", "material_indices", "materials", "bvh", "env", "camera"):
        assert np.array_equal(got[k], want[k], equal_nan=got[k].dtype.kind == "f"), k


def test_big_leaf_goes_through_the_indirection_table(paths):
    biggest, _ = _bvh_shape(R.Scene(paths["big_leaf"]).arrays())
    assert biggest == 80 > 63


def test_deep_chain_reaches_max_bvh_depth(paths):
    _, deepest = _bvh_shape(R.Scene(paths["deep"]).arrays())
    assert deepest == 30             # nodes on the longest root-to-leaf path
