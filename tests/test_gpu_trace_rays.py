"""Traversal parity on caller-chosen rays: rt_trace_rays (the render's trace kernel) against the
oracle's restatement of the sphere loop + bvh_closest_hit_distance (scene.cu:338-372, :134-241).

Besides random rays this drives the corner cases a render reaches only by chance: direction
components that are exactly zero (1/d = inf, so the slab planes give 0 * inf = NaN when the
origin lies on one), axis-aligned rays, origins exactly on triangle vertices (on box faces),
rays that start inside the geometry, and non-finite origins and directions (a NaN hit distance
becomes the next bounce's NaN origin: lamp's glass makes them in a render; the reference then
accepts the first triangle it tests with a NaN t).  Bit-exact t and index (NaN = NaN), exact
traversal counters, through both builds of the kernel (with and without the counters).
"""
import numpy as np
import pytest

import oracle_lib as O
import rtamd as R

pytestmark = pytest.mark.gpu


def _scenes(name, use_bvh=True):
    path = "%s/%s.scene" % (R.ASSETS, name)
    img = (16, 16, 1, 1)
    return O.OracleScene(path, use_bvh=use_bvh, image=img), R.Scene(path, use_bvh=use_bvh, image=img)


def _unit(v):
    v = np.asarray(v, np.float32)
    n = np.sqrt((v * v).sum(-1, keepdims=True)).astype(np.float32)
    return (v / n).astype(np.float32)


def _ray_sets(orc, rng, n):
    arr = orc.arrays()
    tri = arr["triangles"].reshape(-1, 12) if arr["triangles"].size else np.zeros((0, 12), np.float32)
    if tri.shape[0]:
        # triangle storage: p1, p2-p1, p3-p1, normal (scene.cuh:15-26)
        verts = np.concatenate([tri[:, 0:3], tri[:, 0:3] + tri[:, 3:6], tri[:, 0:3] + tri[:, 6:9]])
        lo, hi = verts.min(0), verts.max(0)
    else:
        verts = arr["spheres"].reshape(-1, 4)[:, :3]
        lo, hi = verts.min(0) - 3, verts.max(0) + 3
    span = np.maximum(hi - lo, 1e-3)
    sets = {}
    o = (lo - 0.1 * span + rng.random((n, 3)) * 1.2 * span).astype(np.float32)
    sets["random"] = np.hstack([o, _unit(rng.normal(size=(n, 3)))])
    axes = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    sets["axis_aligned"] = np.hstack([o, axes[rng.integers(0, 6, n)]])
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[np.arange(n), rng.integers(0, 3, n)] = 0.0                     # one exact zero component
    sets["zero_component"] = np.hstack([o, _unit(d)])
    vo = verts[rng.integers(0, len(verts), n)].astype(np.float32)   # origins on vertices / box faces
    sets["vertex_origin"] = np.hstack([vo, _unit(rng.normal(size=(n, 3)))])
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[np.arange(n), rng.integers(0, 3, n)] = 0.0
    sets["vertex_origin_zero_component"] = np.hstack([vo, _unit(d)])
    sets["vertex_origin_axis"] = np.hstack([vo, axes[rng.integers(0, 6, n)]])
    # rays that leave the scene's bounds at once (the oracle: one pop, one internal visit, no triangle
    # test): both of the root's children missed, so they end inside the trace kernel's refill, at the
    # root step it runs there
    c = (lo + hi) / 2
    out = _unit(rng.normal(size=(n, 3)))
    oo = (c + out * (0.5 * np.linalg.norm(span) + 0.01 * rng.random((n, 1)) * span.max())).astype(np.float32)
    sets["outward"] = np.hstack([oo, _unit(out + 0.3 * rng.normal(size=(n, 3)))])
    nf = np.hstack([o, _unit(rng.normal(size=(n, 3)))]).astype(np.float32)
    k = np.arange(n)
    nf[k % 4 == 0, rng.integers(0, 3)] = np.nan                       # NaN origin component
    nf[k % 4 == 1, 3 + rng.integers(0, 3)] = np.nan                   # NaN direction component
    nf[k % 4 == 2, rng.integers(0, 3)] = np.inf                       # infinite origin component
    nf[k % 4 == 3, 3:6] = 0.0                                         # zero direction
    sets["non_finite"] = nf
    return sets


def _same(t_o, i_o, t_g, i_g):
    both_nan = np.isnan(t_o) & np.isnan(t_g)
    return np.nonzero(((t_o.view(np.uint32) != t_g.view(np.uint32)) & ~both_nan) | (i_o != i_g))[0]


@pytest.mark.parametrize("scene,use_bvh", [("cornell", True), ("cornell_plus", True), ("spheres", True),
                                           ("teapot", True), ("lamp_available", True), ("cornell", False)])
def test_trace_rays_bitexact(scene, use_bvh):
    if R.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    orc, dev = _scenes(scene, use_bvh)
    rng = np.random.default_rng(1234)
    for name, rays in _ray_sets(orc, rng, 20000).items():
        t_o, i_o, s_o = orc.closest_hit(rays)
        t_g, i_g, s_g = R.trace_rays(dev, rays, counters=True)
        bad = _same(t_o, i_o, t_g, i_g)
        assert bad.size == 0, "%s/%s: %d rays differ, first %s: oracle (%r, %d) gpu (%r, %d)" % (
            scene, name, bad.size, bad[:1], t_o[bad[0]], i_o[bad[0]], t_g[bad[0]], i_g[bad[0]])
        for k in ("nodes_popped", "internal_visits", "triangle_tests", "sphere_tests"):
            assert s_o[k] == s_g[k], (scene, name, k, s_o[k], s_g[k])
        # the render's build of the kernel (no counters)
        t_r, i_r, _ = R.trace_rays(dev, rays)
        bad = _same(t_o, i_o, t_r, i_r)
        assert bad.size == 0, "%s/%s (render build): %d rays differ" % (scene, name, bad.size)
        assert name in ("non_finite", "outward") or (i_o >= 0).any()


def test_trace_rays_empty_and_single():
    orc, dev = _scenes("cornell")
    t, i, _ = R.trace_rays(dev, np.zeros((0, 6), np.float32))
    assert t.size == 0 and i.size == 0
    ray = np.array([[0.0, 1.0, 3.0, 0.0, 0.0, -1.0]], np.float32)
    t_o, i_o, _ = orc.closest_hit(ray)
    t_g, i_g, _ = R.trace_rays(dev, ray)
    assert t_o.view(np.uint32)[0] == t_g.view(np.uint32)[0] and i_o[0] == i_g[0]
