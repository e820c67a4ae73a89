"""bench.py's N-GPU path with the real HIP renderer at world 2, on the one GPU this box has (round 5).

The driver's SCALE run is bench.run() under torchrun, one process per GPU over RCCL; RCCL refuses two ranks on one
GPU, so here two processes share cuda:0 and the collectives go through gloo with the device tensors staged through
host memory (StagedDist).  Everything else is the product path: RtamdBackend's renderers (librtamd.so), the
overlapped exchange (run_async / wait_pass / finish on each rank's renderer, accumulation off), PassShardedFrame's
slice all-to-all and ordered adds, the gather to rank 0, the weak-scaling frame extension.  The frame assembled in
the timed region must equal the oracle's render of the same frame bit for bit (the reference's pass loop,
raytracing.cu:222-254), and rank 0 alone prints the line."""
import io
import json
import os
import socket
import sys

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = ("teapot.scene", 96, 54, 100, 16, True, True)     # 5 passes of 20 spp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class StagedDist:
    """torch.distributed's calls that bench.py and rtamd_dist make, over gloo, with device tensors copied through
    host memory (gloo's all-to-all and gather take CPU tensors only)."""

    def __init__(self, dist, torch):
        self.d, self.torch = dist, torch
        self.ReduceOp = dist.ReduceOp

    def get_rank(self):
        return self.d.get_rank()

    def get_world_size(self):
        return self.d.get_world_size()

    def barrier(self):
        self.d.barrier()

    def destroy_process_group(self):
        self.d.destroy_process_group()

    def all_reduce(self, t, op=None):
        h = t.cpu()
        self.d.all_reduce(h, op=op if op is not None else self.d.ReduceOp.SUM)
        t.copy_(h)

    def all_to_all_single(self, recv, send):
        h_recv = self.torch.empty(recv.shape, dtype=recv.dtype)
        self.d.all_to_all_single(h_recv, send.cpu())
        recv.copy_(h_recv)

    def gather(self, t, gather_list=None, dst=0):
        h_list = [self.torch.empty(t.shape, dtype=t.dtype) for _ in gather_list] if gather_list is not None else None
        self.d.gather(t.cpu(), gather_list=h_list, dst=dst)
        if gather_list is not None:
            for g, h in zip(gather_list, h_list):
                g.copy_(h)


def _worker(rank, world, port, tmp, steps, golden):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", RTAMD_INFLIGHT="16")
    sys.path[:0] = [REPO, os.path.join(REPO, "cuda-raytracer_amd")]
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)                  # torch's HIP runtime first, then librtamd on it
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    backend = bench.RtamdBackend(use_dist=False)
    backend.world, backend.rank, backend.local = world, rank, 0
    backend.dist, backend.torch, backend.device = StagedDist(dist, torch), torch, torch.device("cuda", 0)
    backend.use_dist = True
    argv = ["--gpus", str(world), "--scene", "teapot", "--warmup", "1", "--no-cpu-baseline"]
    if steps:
        argv += ["--steps", str(steps)]
    buf = io.StringIO()
    res = bench.run(bench.parse_args(argv), backend, cfg=CFG, json_out=buf, golden=golden)
    with open(os.path.join(tmp, "rank%d.json" % rank), "w") as f:
        json.dump({"stdout": buf.getvalue(), "none": res is None}, f)
    if rank == 0:
        np.save(os.path.join(tmp, "fb.npy"), res["timed_fb"])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("steps", [None, 3])
def test_bench_world2_real_renderer(tmp_path, steps):
    import hashlib
    import torch.multiprocessing as mp
    scene_file, W, H, spp, bounces = CFG[:5]
    world = 2
    frame_spp = spp if steps is None or -(-spp // 20) >= world * steps else 20 * world * steps
    osc = O.OracleScene(os.path.join(O.ASSETS, scene_file), image=(W, H, frame_spp, bounces))
    ofb, _ = osc.render(sort=True)
    p0 = O.OracleScene(os.path.join(O.ASSETS, scene_file), image=(W, H, spp, bounces))
    fb0, _ = p0.render(sort=True, pass_begin=0, pass_count=1)
    golden = {"sha256": hashlib.sha256(np.asarray(fb0, dtype="<f4").tobytes()).hexdigest()}
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), steps, golden), nprocs=world, join=True)
    recs = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(world)]
    assert not recs[0]["none"] and recs[1]["none"] and recs[1]["stdout"] == ""
    lines = recs[0]["stdout"].strip().splitlines()
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["config"]["n_ranks_seen"] == world
    assert line["bit_exact_vs_oracle"] is True
    fb = np.load(tmp_path / "fb.npy")
    if steps is None:
        assert np.array_equal(fb, ofb)               # the whole frame, assembled from both ranks' slices
    else:
        # weak scaling: the timed steps are rounds 0..steps-1 of the extended frame: every pass of it here
        assert frame_spp == 20 * world * steps and np.array_equal(fb, ofb)
