"""bench.py's multi-GPU pass sharding (rtamd_dist.PassShardedFrame) over torch.distributed "nccl"
(RCCL) at world 1 on the one-GPU box.

One renderer call per round (max_rounds_per_call=1) makes every call render into buffers that the
previous round's torch work (the stage -> buffer copy, the slice adds) read on torch's stream; the
renderer's own streams do not wait for torch's, so PassShardedFrame synchronises torch's stream
before each call (rtamd_dist.PassShardedFrame._sync).  The frame is rendered twice through the same
buffers and must equal the oracle bit for bit both times.  N > 1 runs the same code with a real
all-to-all; that is covered on the CPU by tests/test_multigpu_gloo.py (world 2, 3, 5)."""
import os
import socket

import numpy as np
import pytest

import oracle_lib as O
import rtamd as R
import rtamd_dist as D

pytestmark = pytest.mark.gpu

IMAGE = (64, 48, 100, 6)          # 5 passes


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def rccl():
    import torch
    import torch.distributed as dist
    if R.device_count() < 1 or not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    yield torch, dist
    dist.destroy_process_group()


class AsyncPasses:
    """bench.py's asynchronous renderer adapter: rt_renderer_run_async / wait_pass / finish."""

    def __init__(self, ren, torch):
        self.ren, self.torch = ren, torch

    def start(self, passes, out):
        stride = passes[1] - passes[0] if len(passes) > 1 else 1
        self.ren.run_async(passes[0], len(passes), stride, out.data_ptr())

    def wait(self, j):
        self.ren.wait_pass(j, self.torch.cuda.current_stream().cuda_stream)

    def finish(self):
        self.ren.finish()


@pytest.mark.parametrize("sort", [True, False])
@pytest.mark.parametrize("chunk,xrounds", [(1, None), (2, None), (None, None), (None, 1), (None, 2), (2, 1)])
def test_pass_sharded_frame_rccl_world1(rccl, sort, chunk, xrounds):
    """xrounds: the overlapped exchange (rt_renderer_run_async; torch's stream waits on per-pass events
    and adds the slices of every xrounds rounds while later passes render)."""
    torch, dist = rccl
    path = "%s/cornell_plus.scene" % R.ASSETS
    ref, _ = O.OracleScene(path, image=IMAGE).render(sort=sort)
    psc = R.Scene(path, image=IMAGE)
    ren = R.Renderer(psc, sort=sort)
    try:
        def render_passes(passes, out):
            stride = passes[1] - passes[0] if len(passes) > 1 else 1
            ren.run(pass_begin=passes[0], count=len(passes), stride=stride, d_pass_sums=out.data_ptr())

        frame = D.PassShardedFrame(dist, torch, psc.pixels * 3, psc.passes, torch.device("cuda", 0), render_passes,
                                   max_rounds_per_call=chunk, async_render=AsyncPasses(ren, torch) if xrounds else None,
                                   exchange_rounds=xrounds or 4)
        for attempt in range(2):            # the second frame reuses every buffer of the first
            frame.reset()
            assert frame.run_all() == psc.passes
            got = frame.fb.cpu().numpy()
            assert np.array_equal(got, ref), "frame %d differs from the oracle" % attempt
    finally:
        ren.close()
