"""GPU parity on the synthetic edge-case scenes (tests/edge_scenes.py), through the C ABI:

* big_leaf: an 80-triangle leaf (indirection-table leaf ref) -- closest hits on rays aimed at
  it and full renders, sort on and off;
* deep: a 30-level chain.  Rays along -x through the hole every triangle leaves around the x
  axis push one near child per level (the reference's far-child-first order, scene.cu:204-225),
  so the trace kernel's stack spills past its 8 LDS entries into the global overflow and back.
Bit-exact t, hit index and traversal counters against the oracle; renders bit-exact."""
import numpy as np
import pytest

import edge_scenes
import oracle_lib as O
import rtamd as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def paths(tmp_path_factory):
    if R.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    return edge_scenes.write(str(tmp_path_factory.mktemp("edge")))


def _unit(v):
    v = np.asarray(v, np.float32)
    return (v / np.sqrt((v * v).sum(-1, keepdims=True)).astype(np.float32)).astype(np.float32)


def _check_trace(path, rays):
    rays = np.ascontiguousarray(rays, np.float32)
    osc, psc = O.OracleScene(path), R.Scene(path)
    ot, oi, ost = osc.closest_hit(rays)
    gt, gi, gst = R.trace_rays(psc, rays, counters=True)
    assert np.array_equal(gi, oi)
    assert np.array_equal(gt.view(np.uint32), ot.view(np.uint32))
    for k in ("nodes_popped", "internal_visits", "triangle_tests"):
        assert gst[k] == ost[k], k
    return gi, ost


def test_deep_chain_axis_rays(paths):
    rng = np.random.default_rng(11)
    n = 4096
    yz = (rng.random((n, 2)) * 0.2 - 0.1).astype(np.float32)       # inside every triangle's hole
    o = np.hstack([np.full((n, 1), 1e29, np.float32), yz])
    d = np.tile(np.array([[-1, 0, 0]], np.float32), (n, 1))
    idx, st = _check_trace(paths["deep"], np.hstack([o, d]))
    assert (idx == -1).all()                                         # nothing hit...
    assert st["internal_visits"] >= 29 * n                            # ...after walking the whole chain
    assert st["max_stack"] > 8                                        # past the LDS part of the stack
    # from the near end towards +x, and oblique rays that do hit triangles
    o2 = np.hstack([np.full((n, 1), -5.0, np.float32), yz])
    d2 = np.tile(np.array([[1, 0, 0]], np.float32), (n, 1))
    o3 = (rng.random((n, 3)) * np.array([1e12, 4, 4]) - np.array([0, 2, 2])).astype(np.float32)
    d3 = _unit(np.hstack([-np.ones((n, 1)), rng.normal(size=(n, 2)) * 1e-3]))
    _check_trace(paths["deep"], np.vstack([np.hstack([o2, d2]), np.hstack([o3, d3])]))


def test_big_leaf_rays(paths):
    rng = np.random.default_rng(12)
    n = 4096
    o = np.hstack([np.full((n, 1), -4.0), rng.random((n, 2)) * [1.6, 1.6] + [0.2, -0.8]]).astype(np.float32)
    d = _unit(np.hstack([np.ones((n, 1)), rng.normal(size=(n, 2)) * 0.05]))
    idx, _ = _check_trace(paths["big_leaf"], np.hstack([o, d]))
    assert ((idx >= 0) & (idx < 80)).sum() > n // 4                  # many hits inside the big leaf


@pytest.mark.parametrize("name", ["big_leaf", "deep"])
@pytest.mark.parametrize("sort", [True, False])
def test_edge_scene_render_bitexact(paths, name, sort):
    osc, psc = O.OracleScene(paths[name]), R.Scene(paths[name])
    ofb, ost = osc.render(sort=sort)
    gfb, gst = R.render(psc, sort=sort, counters=True)
    assert np.array_equal(gfb, ofb)
    assert gst["live_segments"] == ost["live_segments"]
    assert gst["nodes_popped"] == ost["nodes_popped"]


def test_bvh_deeper_than_the_stack_is_refused(paths):
    """A caller-supplied BVH (rt_scene.bvh, e.g. through the reference-side binding of
    INTEGRATION.md) deeper than the trace kernel's 32-entry stack is refused with RT_E_INVALID
    instead of running past the per-lane overflow stack.  The loader caps depth at the
    reference's MAX_BVH_DEPTH 30 (scene.cu:10), so the chain is built by hand: internal node
    2k+1 has children (2k+3, 2k+4), 2k+4 an empty leaf."""
    import ctypes as C
    psc = R.Scene(paths["deep"])
    for levels, ok in ((31, True), (40, False)):
        nodes = np.zeros((2 * levels + 1, 8), np.float32)
        ints = nodes.view(np.int32)
        nodes[:, 0:3], nodes[:, 3:6] = -1e30, 1e30
        ints[0, 6:8] = (1, 2)                       # root: children 1 (internal), 2 (empty leaf)
        for k in range(levels - 1):
            ints[2 * k + 1, 6:8] = (2 * k + 3, 2 * k + 4)
        # leaves: child2 <= child1 (empty: 0, 0); the deepest internal node's children are leaves
        v = psc.view
        saved = (v.bvh, v.bvh_node_count)
        v.bvh, v.bvh_node_count = nodes.ctypes.data, nodes.shape[0]
        try:
            rays = np.array([[0, 0, 0, 1, 0, 0]], np.float32)
            if ok:
                R.trace_rays(psc, rays)
            else:
                with pytest.raises(R.RtError, match="deeper"):
                    R.trace_rays(psc, rays)
                # the multi-device render (rt_multi.hip): a device whose setup fails returns the
                # error through the setup barrier instead of entering a collective
                with pytest.raises(R.RtError, match="deeper"):
                    R.render(psc, devices=[0])
        finally:
            v.bvh, v.bvh_node_count = saved
