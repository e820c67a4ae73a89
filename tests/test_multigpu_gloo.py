"""N>1 path on CPU: gloo process groups (world 2, 3, 5) running the same pass-sharding,
pixel-slice all-to-all and ordered per-slice accumulation (rtamd_dist.PassShardedFrame) that
bench.py runs over RCCL.  Pass sums come from the oracle here (the GPU renders them on the box);
the assembled frame must be bit-identical to the single-process render.  World 5 does not divide
W*H*3 = 1152, so it covers the padded-slice path; chunk 2 covers several exchanges per frame."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
import rtamd_dist as D

IMAGE = (24, 16, 100, 4)       # 5 passes: uneven over 2 ranks


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class LazyAsyncRender:
    """The asynchronous renderer's contract (rtamd.Renderer.run_async / wait_pass / finish) with the
    oracle's pass sums, each rendered only when the frame waits for that pass (or at finish): a pass
    the frame used before waiting for it would still be zeros, and the frame would not be exact."""

    def __init__(self, sc):
        self.sc, self.todo = sc, {}

    def start(self, passes, out):
        out.zero_()
        self.todo = {j: (p, out[j]) for j, p in enumerate(passes)}

    def wait(self, j):
        p, row = self.todo.pop(j, (None, None))
        if p is not None:
            row.copy_(torch.from_numpy(self.sc.pass_sums(sort=True, pass_begin=p, pass_count=1, threads=2)[0]))

    def finish(self):
        for j in list(self.todo):
            self.wait(j)


def _worker(rank, world, port, out_path, chunk, xrounds=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = O.OracleScene(os.path.join(O.ASSETS, "cornell_plus.scene"), image=IMAGE)

    def render_passes(passes, out):
        for j, p in enumerate(passes):
            out[j].copy_(torch.from_numpy(sc.pass_sums(sort=True, pass_begin=p, pass_count=1, threads=2)[0]))

    frame = D.PassShardedFrame(dist, torch, sc.pixels * 3, sc.passes, "cpu", render_passes, max_rounds_per_call=chunk,
                               async_render=LazyAsyncRender(sc) if xrounds else None, exchange_rounds=xrounds or 4)
    n = frame.run_all()
    assert n == len(D.pass_schedule(rank, world, sc.passes))
    if rank == 0:
        np.save(out_path, frame.fb.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunk,xrounds", [(2, 2, None), (3, None, None), (5, None, None),
                                                 (2, None, 1), (3, 2, 1), (2, None, 2), (8, None, None)])
def test_pass_sharded_frame_is_bitexact(tmp_path, world, chunk, xrounds):
    """xrounds: the overlapped exchange (an asynchronous renderer, slices exchanged every xrounds rounds)."""
    out = str(tmp_path / "fb.npy")
    mp.spawn(_worker, args=(world, _free_port(), out, chunk, xrounds), nprocs=world, join=True)
    got = np.load(out)
    ref, _ = O.OracleScene(os.path.join(O.ASSETS, "cornell_plus.scene"), image=IMAGE).render(sort=True)
    assert np.array_equal(got, ref)


def test_schedule_covers_every_pass_once():
    for world in (1, 2, 3, 8):
        for passes in (1, 5, 103, 205):
            got = sorted(p for r in range(world) for p in D.pass_schedule(r, world, passes))
            assert got == list(range(passes))


def _tile_worker(rank, world, port, out_path, rows):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = O.OracleScene(os.path.join(O.ASSETS, "cornell_plus.scene"), image=IMAGE)
    W, H = IMAGE[0], IMAGE[1]

    def render_tile(out):
        # the tile render equals the full render on the owned rows and is 0 elsewhere
        # (tests/test_gpu_tiles.py checks that of the HIP path); the oracle stands in for it here
        full = sc.render(sort=False, threads=2)[0].reshape(H, W * 3)
        mask = np.zeros((H, 1), np.float32)
        mask[D.tile_rows(H, world, rank, rows)] = 1
        out.copy_(torch.from_numpy(full * mask))

    frame = D.TileShardedFrame(dist, torch, W, H, "cpu", render_tile, rows=rows)
    fb = frame.run_all()
    if rank == 0:
        np.save(out_path, fb.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,rows", [(2, 8), (3, 3), (4, 8)])   # (4, 8): 2 stripes, ranks 2-3 own none
def test_tile_sharded_frame_is_bitexact(tmp_path, world, rows):
    out = str(tmp_path / "fb.npy")
    mp.spawn(_tile_worker, args=(world, _free_port(), out, rows), nprocs=world, join=True)
    got = np.load(out)
    ref, _ = O.OracleScene(os.path.join(O.ASSETS, "cornell_plus.scene"), image=IMAGE).render(sort=False)
    assert np.array_equal(got, ref)


def test_tile_rows_cover_the_image_once():
    for world in (1, 2, 3, 8):
        for h, rows in ((1080, 8), (512, 8), (17, 3), (5, 8)):
            got = sorted(y for r in range(world) for y in D.tile_rows(h, world, r, rows))
            assert got == list(range(h))


def _tile_sort_worker(rank, world, port, out_path, scene, image, rows, sort):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = O.OracleScene(os.path.join(O.ASSETS, scene + ".scene"), image=image)
    fb, st = sc.render_tiled(D.bucket_exchange(dist, torch), world, rank, tile_rows=rows, sort=sort, threads=2)
    t = torch.from_numpy(fb)
    dist.reduce(t, dst=0)                   # owners' pixels are disjoint, the rest 0: x + 0 = x exactly
    live = torch.tensor([st["live_segments"]], dtype=torch.int64)
    dist.reduce(live, dst=0)
    if rank == 0:
        np.save(out_path, t.numpy())
        np.save(out_path + ".live.npy", live.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,scene,image,rows,sort", [
    (2, "cornell_plus", (24, 16, 45, 5), 3, True),    # 3 passes, short last pass, 3-row stripes
    (3, "teapot", (40, 22, 20, 8), 8, True),          # BVH + env map; 22 rows: a short last stripe
    (2, "spheres", (20, 12, 20, 6), 4, True),
    (2, "cornell", (24, 16, 20, 4), 5, False)])       # sort off: no exchange, slot = ray index
def test_tile_sharded_sort_on_is_bitexact(tmp_path, world, scene, image, rows, sort):
    """Pixel tiles WITH the reorder on: each owner renders only its stripes; after
    every bounce but the last the owners all-reduce one byte per live ray (bucket + 1 at its global
    slot) over gloo and rank their own rays by the global stable order, so every process seed is
    the one the single-GPU render uses (raytracing.cu:89 after :238-247).  The assembled frame and
    the live segment count equal the single-process oracle render bit for bit."""
    out = str(tmp_path / "fb.npy")
    mp.spawn(_tile_sort_worker, args=(world, _free_port(), out, scene, image, rows, sort), nprocs=world, join=True)
    ref, rst = O.OracleScene(os.path.join(O.ASSETS, scene + ".scene"), image=image).render(sort=sort)
    assert np.array_equal(np.load(out), ref)
    assert int(np.load(out + ".live.npy")[0]) == rst["live_segments"]
