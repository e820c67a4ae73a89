"""bench.py's own N-GPU orchestration, run end to end over gloo on CPU (world 2, 4 and 8).

bench.run() is the code the driver's SCALE run executes on every rank (torchrun, one process per
GPU): the weak-scaling frame extension, the rank-0-only legs (exclusive pass, parity hash), the
warmup / timed / event-timed / counted / full-frame legs with their collectives, reduce(),
n_ranks_seen and the one JSON line on rank 0.  Here its renderer and collectives come from a test
backend: the oracle's pass sums (tests/oracle_lib.py) stand in for the HIP renderer, gloo for
RCCL, exactly as tests/test_multigpu_gloo.py drives rtamd_dist.  The frame assembled in the timed
region must equal the single-process oracle render bit for bit (the reference's pass loop,
raytracing.cu:222-254), and rank 0 alone prints the line."""
import ctypes
import io
import json
import os
import socket
import sys
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = ("cornell_plus.scene", 24, 16, 60, 4, True, True)   # 3 passes of 20 spp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class OracleRenderer:
    """rtamd.Renderer's interface over the oracle: run() renders each pass alone (0 + S_p = the pass
    sum, exactly) and stores the sums at d_pass_sums (a CPU tensor's data pointer here)."""

    def __init__(self, sc, sort):
        self.sc, self.sort = sc, sort
        self.px3 = sc.pixels * 3

    def run(self, pass_begin=0, count=1, stride=1, d_pass_sums=None):
        out = None
        if d_pass_sums:
            out = np.ctypeslib.as_array((ctypes.c_float * (count * self.px3)).from_address(d_pass_sums))
        acc = {}
        for j in range(count):
            fb, st = self.sc.render(sort=self.sort, pass_begin=pass_begin + stride * j, pass_count=1, threads=2)
            if out is not None:
                out[j * self.px3:(j + 1) * self.px3] = fb
            st["hits"] = st["hits_triangle"] + st["hits_sphere"]   # rt_stats' names
            for k, v in st.items():
                acc[k] = acc.get(k, 0) + int(v)
        acc.update(trace_ms=0.0, trace_launches=0, process_ms=0.0, sort_ms=0.0, kernel_ms=0.0)
        return acc

    def set_event_timing(self, on):
        pass

    def set_counters(self, on):
        pass

    def clear(self):
        pass

    def close(self):
        pass


class OracleBackend:
    def __init__(self, log):
        self.dist, self.torch = dist, torch
        self.world, self.rank, self.local = dist.get_world_size(), dist.get_rank(), 0
        self.device = torch.device("cpu")
        self.log = log

    def scene(self, scene_file, use_bvh, image):
        sc = O.OracleScene(os.path.join(O.ASSETS, scene_file), use_bvh=use_bvh, image=image)
        i = sc.info
        sc.view = types.SimpleNamespace(bvh_node_count=i.bvh_node_count, triangle_count=i.triangle_count,
                                        sphere_count=i.sphere_count)
        sc.bvh_ms = 0.0
        return sc

    def renderer(self, scene, sort, tiles):
        assert tiles is None
        return OracleRenderer(scene, sort)

    def exclusive_pass(self, scene, sort):
        self.log.append("exclusive_pass")
        _, st = scene.render(sort=sort, pass_begin=0, pass_count=1, threads=2)
        return {"trace_ms": 1.0, "launches": 4, "ms_per_launch": 0.25, "kernel_ms": 1.0, "launch_profile": [],
                "counted": {k: int(v) for k, v in st.items()}}

    def render_pass0(self, scene, sort):
        self.log.append("render_pass0")
        return scene.render(sort=sort, pass_begin=0, pass_count=1, threads=2)[0]

    def barrier_sync(self):
        dist.barrier()


def _worker(rank, world, port, tmp, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, REPO)
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    log = []
    argv = ["--gpus", str(world), "--scene", "cornell_plus", "--warmup", "1"]
    if steps:
        argv += ["--steps", str(steps)]
    args = bench.parse_args(argv)
    buf = io.StringIO()
    res = bench.run(args, OracleBackend(log), cfg=CFG, json_out=buf)
    with open(os.path.join(tmp, "rank%d.json" % rank), "w") as f:
        json.dump({"stdout": buf.getvalue(), "log": log, "none": res is None}, f)
    if rank == 0:
        np.save(os.path.join(tmp, "fb.npy"), res["timed_fb"])
    dist.barrier()
    dist.destroy_process_group()


# (8, 1): the driver's SCALE shape at N = 8 (one rank per GPU, weak-scaling frame extension)
@pytest.mark.parametrize("world,steps", [(2, None), (4, None), (2, 2), (4, 1), (8, 1)])
def test_bench_run_over_gloo(tmp_path, world, steps):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), steps), nprocs=world, join=True)
    recs = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(world)]
    # one JSON line, on rank 0 only; the rank-0-only legs ran on rank 0 only
    assert not recs[0]["none"] and all(r["none"] for r in recs[1:])
    assert all(r["stdout"] == "" for r in recs[1:])
    lines = recs[0]["stdout"].strip().splitlines()
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert recs[0]["log"] == ["exclusive_pass", "render_pass0"]
    assert all(r["log"] == [] for r in recs[1:])
    cfgd = line["config"]
    assert cfgd["n_ranks_seen"] == world and line["n_gpus"] == world
    assert cfgd["passes_in_flight"]["cap"] == 16      # next to RCCL (bench.py's RTAMD_INFLIGHT)
    W, H, spp, bounces = CFG[1:5]
    if steps is None:
        frame_spp = spp
        assert line["scaling"] == "strong" and line["steps"] == -(-3 // world)
        assert "frame_extended" not in cfgd
    else:
        frame_spp = max(spp, 20 * world * steps)
        assert line["scaling"] == "weak" and line["steps"] == steps
        assert ("frame_extended" in cfgd) == (frame_spp != spp)
    assert cfgd["passes_per_frame"] == -(-frame_spp // 20)
    assert line["bit_exact_vs_oracle"] is None or isinstance(line["bit_exact_vs_oracle"], bool)
    assert line["render_wall_ms"] and line["value"] > 0
    # the timed region's frame: every pass of the (extended) frame, assembled from the ranks' pixel
    # slices, equals one process's render bit for bit
    got = np.load(tmp_path / "fb.npy")
    ref, _ = O.OracleScene(os.path.join(O.ASSETS, CFG[0]), image=(W, H, frame_spp, bounces)).render(sort=True,
                                                                                                   threads=2)
    assert np.array_equal(got, ref)


class OracleMulti:
    """rtamd.MultiRenderer's interface over the oracle (the in-library backend without torchrun): run(n)
    renders passes 0..n-1 of the frame, dealt round-robin over the `devices`, each device adding its passes'
    sums into its own slice of the frame in pass order as rt_multi's owners do -- here every pass is
    rendered alone and added in pass order, which is that per-pixel sequence."""

    def __init__(self, sc, sort, devices):
        self.sc, self.sort, self.devices = sc, sort, devices
        self.fb = None
        self.ranks = devices

    def run(self, pass_count=-1):
        P = self.sc.passes if hasattr(self.sc, "passes") else None
        n = pass_count if pass_count >= 0 else P
        fb = np.zeros(self.sc.pixels * 3, np.float32)
        acc = {}
        for p in range(n):
            pf, st = self.sc.render(sort=self.sort, pass_begin=p, pass_count=1, threads=2)
            fb = fb + pf
            st["hits"] = st["hits_triangle"] + st["hits_sphere"]
            for k, v in st.items():
                acc[k] = acc.get(k, 0) + int(v)
        self.fb = fb
        acc.update(trace_ms=0.0, trace_launches=0, process_ms=0.0, sort_ms=0.0, kernel_ms=0.0, passes=n)
        return acc

    def framebuffer(self):
        return self.fb

    def set_event_timing(self, on):
        pass

    def set_counters(self, on):
        pass

    def close(self):
        pass


class OracleInLibBackend(OracleBackend):
    inlib = True

    def __init__(self, log, n):
        self.dist = self.torch = None
        self.world, self.rank, self.local = n, 0, 0
        self.device = None
        self.use_dist = False
        self.log = log

    def renderer(self, scene, sort, tiles):
        assert tiles is None
        return OracleMulti(scene, sort, self.world)

    def barrier_sync(self):
        pass


@pytest.mark.parametrize("n,steps", [(2, None), (3, 1)])
def test_bench_run_in_library_backend(n, steps, monkeypatch):
    """`--gpus N` without torchrun (WORLD_SIZE unset): bench.run over the in-library backend (one process,
    rt_multi over N GPUs; here the oracle stands in) reports n_gpus == n_ranks_seen == N, and the timed
    frame equals the single-process render bit for bit."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    sys.path.insert(0, REPO)
    import bench
    args = bench.parse_args(["--gpus", str(n), "--scene", "cornell_plus", "--warmup", "1", "--no-cpu-baseline"] +
                            (["--steps", str(steps)] if steps else []))
    log = []
    buf = io.StringIO()
    res = bench.run(args, OracleInLibBackend(log, n), cfg=CFG, json_out=buf)
    line = json.loads(buf.getvalue().strip())
    assert line["n_gpus"] == n and line["config"]["n_ranks_seen"] == n
    assert "rt_multi" in line["config"]["launch"]
    W, H, spp, bounces = CFG[1:5]
    frame_spp = spp if steps is None else max(spp, 20 * n * steps)
    assert line["steps"] == (-(-3 // n) if steps is None else steps)
    if steps is None:
        ref, _ = O.OracleScene(os.path.join(O.ASSETS, CFG[0]), image=(W, H, frame_spp, bounces)).render(
            sort=True, threads=2)
        assert np.array_equal(res["timed_fb"], ref)
    assert res["my_passes"] == -(-frame_spp // 20)


def test_bench_gpus_argument_is_checked():
    """--gpus N is never ignored: WORLD_SIZE (torchrun) must equal it, and without torchrun N may not exceed
    the visible HIP devices (none in this container): both exit with status 2 before any rendering."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--no-extras"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "HIP device(s) visible" in r.stderr, r.stderr[-2000:]
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "3", "--no-extras"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr, r.stderr[-2000:]
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--no-extras"],
                       env=dict(env, RTAMD_HW_QUEUES="40"), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "1..32" in r.stderr
