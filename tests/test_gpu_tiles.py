"""Pixel-tile sharding (rt_opts.tile_*): a render restricted to one owner's row
stripes, with sort off, equals the whole-image render on those rows bit for bit and leaves the
other rows 0, so the owners' images add up to the 1-GPU image exactly.  With sort on the process
seeds follow the global post-sort slots (raytracing.cu:89): the owners exchange one byte per
global live ray per bounce (rt_renderer_set_exchange), and without an exchange the render fails."""
import numpy as np
import pytest

import oracle_lib as O
import rtamd as R

pytestmark = pytest.mark.gpu

CASES = [
    # scene, image (W, H, spp, bounces), tile_count, tile_rows
    ("cornell", (64, 64, 24, 4), 3, 8),
    ("teapot", (96, 54, 20, 16), 2, 8),        # 54 rows: the last stripe is 6 rows
    ("lamp_available", (80, 45, 20, 32), 4, 5),
    ("spheres", (33, 17, 7, 1), 5, 2),         # odd sizes, partial pass, short last stripe
    ("cornell_plus", (48, 20, 20, 8), 4, 8),   # 3 stripes over 4 owners: owner 3 has none
]


@pytest.fixture(scope="module")
def gpu():
    if R.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    return 0


@pytest.mark.parametrize("scene,image,count,rows", CASES)
def test_tile_shares_equal_full_render(gpu, scene, image, count, rows):
    path = "%s/%s.scene" % (R.ASSETS, scene)
    psc = R.Scene(path, image=image)
    W, H = image[0], image[1]
    full, fst = R.render(psc, sort=False)
    total = np.zeros_like(full)
    gen = live = 0
    for i in range(count):
        fb, st = R.render(psc, sort=False, tiles=(count, i, rows))
        img = fb.reshape(H, W, 3)
        mine = R.tile_rows_of(H, count, i, rows)
        other = sorted(set(range(H)) - set(mine))
        assert np.array_equal(img[mine], full.reshape(H, W, 3)[mine])
        assert not img[other].any()
        total += fb                              # x + 0 = x: the owners' images add exactly
        gen += st["generated_rays"]
        live += st["live_segments"]
    assert np.array_equal(total, full)
    assert gen == fst["generated_rays"]
    assert live == fst["live_segments"]


def test_tile_share_matches_oracle_rows(gpu):
    path = "%s/teapot.scene" % R.ASSETS
    image = (96, 54, 20, 16)
    ofb, _ = O.OracleScene(path, image=image).render(sort=False)
    fb, _ = R.render(R.Scene(path, image=image), sort=False, tiles=(3, 1, 8))
    rows = R.tile_rows_of(54, 3, 1, 8)
    assert np.array_equal(fb.reshape(54, 96, 3)[rows], ofb.reshape(54, 96, 3)[rows])


def test_tile_renderer_passes_in_flight(gpu):
    # the persistent renderer with several passes in flight, and stride-sharded passes
    path = "%s/teapot.scene" % R.ASSETS
    image = (64, 40, 100, 8)
    psc = R.Scene(path, image=image)
    full, _ = R.render(psc, sort=False)
    ren = R.Renderer(psc, sort=False, tiles=(2, 0, 8))
    ren.run(0, psc.passes, 1)
    fb = ren.framebuffer()
    ren.close()
    rows = R.tile_rows_of(40, 2, 0, 8)
    assert np.array_equal(fb.reshape(40, 64, 3)[rows], full.reshape(40, 64, 3)[rows])


def test_tiles_with_sort_on_need_an_exchange(gpu):
    psc = R.Scene("%s/cornell.scene" % R.ASSETS, image=(32, 32, 4, 2))
    with pytest.raises(R.RtError, match="exchange"):
        R.render(psc, sort=True, tiles=(2, 0))
    with pytest.raises(R.RtError, match="tile_index"):
        R.render(psc, sort=False, tiles=(2, 2))


SORT_ON_CASES = [("cornell_plus", (48, 40, 45, 6), 8, 2),
                 ("teapot", (64, 36, 20, 16), 4, 3),
                 ("spheres", (40, 24, 20, 8), 8, 2),
                 ("lamp_available", (48, 27, 20, 32), 4, 3),
                 ("cornell", (24, 16, 8, 4), 8, 3)]      # 2 stripes, 3 owners: owner 2 has none


def render_owners(path, image, rows, owners, exchange):
    """`owners` tile renderers on this GPU, one per tile owner, each in its own thread, with sort on;
    exchange = "host" (a numpy sum through the host-buffer callback) or "device" (the device-side
    group sum of tests/native/xchg.hip on the pass streams, the stream contract of the library's
    RCCL path).  Returns the owners' framebuffers summed (disjoint pixels) and their stats."""
    import threading
    import xchg_lib
    sc = R.Scene(path, image=image)
    bar = threading.Barrier(owners, timeout=60)
    parts, out, errs = {}, {}, []
    group = xchg_lib.Group(owners) if exchange == "device" else None

    def exchange_for(i):
        def ex(arr):
            parts[i] = arr.copy()
            bar.wait()
            tot = sum(parts[k].astype(np.int32) for k in range(owners))
            bar.wait()
            arr[:] = tot.astype(np.uint8)
        return ex

    def run(i):
        try:
            r = R.Renderer(sc, sort=True, tiles=(owners, i, rows))
            if group:
                group.attach(r, i)
            else:
                r.set_exchange(exchange_for(i))
            st = r.run(pass_begin=0, count=-1)
            out[i] = (r.framebuffer(), st)
            r.close()
        except Exception as e:      # a failed owner would leave the others at the barrier
            errs.append(e)
            bar.abort()
    th = [threading.Thread(target=run, args=(i,)) for i in range(owners)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    if group:
        group.close()
    assert not errs, errs
    fb = sum(out[i][0] for i in range(owners))
    return fb, [out[i][1] for i in range(owners)]


@pytest.mark.parametrize("exchange", ["host", "device"])
@pytest.mark.parametrize("scene,image,rows,owners", SORT_ON_CASES)
def test_tiles_with_sort_on_bitexact(gpu, scene, image, rows, owners, exchange):
    """Pixel tiles WITH the reorder on: `owners` renderers on this GPU exchange one byte
    per global live ray after every bounce but the last (rt_renderer_set_exchange) and rank their
    rays by the global stable order.  Their framebuffers (disjoint pixels) add up to the oracle's
    single-process render bit for bit, and the live segment counts add up to the oracle's.  The
    "device" exchange runs on the pass streams with the renderer waiting only for the live-count
    copy of the previous bounce (rt_render.hip tsort_back), as the RCCL exchange does."""
    path = "%s/%s.scene" % (R.ASSETS, scene)
    ref, rst = O.OracleScene(path, image=image).render(sort=True)
    fb, sts = render_owners(path, image, rows, owners, exchange)
    assert np.array_equal(fb, ref)
    assert sum(s["live_segments"] for s in sts) == rst["live_segments"]


def test_tiles_with_sort_on_all_passes_together(gpu, monkeypatch):
    """RTAMD_TSTAGGER=0: every context's first pass starts at step 0 (no staggering); same image."""
    monkeypatch.setenv("RTAMD_TSTAGGER", "0")
    path = "%s/teapot.scene" % R.ASSETS
    image = (40, 24, 65, 8)
    ref, _ = O.OracleScene(path, image=image).render(sort=True)
    fb, _ = render_owners(path, image, 4, 2, "device")
    assert np.array_equal(fb, ref)


@pytest.mark.parametrize("sort", [True, False])
def test_library_tile_shard_one_device(gpu, sort):
    """rt_render with device_count = 1 and shard_tiles = 1 (rt_multi.hip run_device_tiles: the RCCL
    communicator, the renderer, the ncclReduce of the framebuffer) equals the oracle bit for bit."""
    path = "%s/teapot.scene" % R.ASSETS
    image = (48, 30, 45, 8)
    ref, _ = O.OracleScene(path, image=image).render(sort=sort)
    fb, st = R.render(R.Scene(path, image=image), sort=sort, devices=[0], shard_tiles=True)
    assert np.array_equal(fb, ref)
    assert st["passes"] == 3


@pytest.mark.parametrize("shard_tiles", [False, True])
def test_multi_device_failure_after_setup_returns(gpu, monkeypatch, shard_tiles):
    """A device failing after the setup barrier (RTAMD_FAIL_AFTER_SETUP, a hook of the test build
    librtamd_test.so) makes rt_render return its error; the device aborts only its own communicator
    (no call can race the abort).  The product library ignores the variable."""
    monkeypatch.setenv("RTAMD_FAIL_AFTER_SETUP", "0")
    psc = R.Scene("%s/cornell.scene" % R.ASSETS, image=(32, 32, 8, 2))
    T = R.test_lib()
    with pytest.raises(R.RtError, match="injected failure"):
        R.render(psc, sort=True, devices=[0], shard_tiles=shard_tiles, L=T)
    fb, _ = R.render(psc, sort=True, devices=[0], shard_tiles=shard_tiles)   # no hook in the product
    monkeypatch.delenv("RTAMD_FAIL_AFTER_SETUP")
    fb, _ = R.render(psc, sort=True, devices=[0], shard_tiles=shard_tiles, L=T)   # the library still works
    ref, _ = O.OracleScene("%s/cornell.scene" % R.ASSETS, image=(32, 32, 8, 2)).render(sort=True)
    assert np.array_equal(fb, ref)


@pytest.mark.parametrize("scene,image", [("teapot", (40, 24, 45, 8)), ("lamp_available", (32, 18, 20, 32))])
def test_rccl_exchange_one_rank(gpu, scene, image):
    """rt_rccl_unique_id + rt_renderer_set_exchange_rccl with sort on: owner 0 of a 2-owner split whose
    stripes cover the whole image (one stripe of H rows; owner 1 has none) joins a one-rank RCCL
    communicator, so every per-bounce exchange runs the library's in-place ncclAllReduce on the pass
    stream (an identity sum at one rank) and the render equals the oracle's bit for bit.  RCCL refuses
    two ranks on one GPU, so this is the RCCL exchange's reach on a one-GPU box."""
    path = "%s/%s.scene" % (R.ASSETS, scene)
    W, H = image[0], image[1]
    ref, rst = O.OracleScene(path, image=image).render(sort=True)
    uid = R.rccl_unique_id()
    assert len(uid) == R.RCCL_ID_BYTES
    r = R.Renderer(R.Scene(path, image=image), sort=True, tiles=(2, 0, H))
    r.set_exchange_rccl(uid, 1, 0)
    st = r.run(pass_begin=0, count=-1)
    fb = r.framebuffer()
    r.close()
    assert np.array_equal(fb, ref)
    assert st["live_segments"] == rst["live_segments"]
