"""rt_multi, the persistent in-library multi-GPU renderer (round 6), and bench.py --gpus N without torchrun.

The communicator, one renderer per device and the exchange buffers are set up once; every rt_multi_run renders
the first pass_count passes of the frame round-robin over the devices, exchanges the pass sums as pixel slices and
gathers the frame on the first device (raytracing.cu:222-254's pass loop, sharded).  On this one-GPU box: N = 1
through RCCL with the product library, and N = 2 / 3 through the test build's loopback transport (librtamd_test.so,
RTAMD_MULTI_LOOPBACK=1: the N device threads share the GPU, the two collectives become device copies).  Every frame
must equal the oracle's bit for bit."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as O
import rtamd as R

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _scenes(name, image):
    path = "%s/%s.scene" % (R.ASSETS, name)
    return O.OracleScene(path, image=image), R.Scene(path, image=image)


@pytest.mark.parametrize("sort", [True, False])
def test_multi_renderer_one_device_rccl(sort):
    """N = 1 over RCCL (the product library): reused across runs of part of the frame and the whole frame."""
    osc, psc = _scenes("teapot", (64, 36, 100, 8))      # 5 passes
    m = R.MultiRenderer(psc, [0], sort=sort)
    try:
        assert m.ranks == 1
        for n in (2, -1, 5):
            fb, st = m.run(n, host=True)
            ref, ost = osc.render(sort=sort, pass_begin=0, pass_count=5 if n < 0 else n)
            assert np.array_equal(fb, ref)
            assert st["live_segments"] == ost["live_segments"] and st["passes"] == (5 if n < 0 else n)
        assert np.array_equal(m.framebuffer(), fb)
    finally:
        m.close()


@pytest.mark.parametrize("world,scene,image,sort", [(2, "teapot", (64, 36, 100, 16), True),
                                                    (3, "cornell_plus", (40, 32, 350, 5), True),
                                                    (2, "cornell", (33, 17, 190, 4), False)])
def test_multi_renderer_loopback(monkeypatch, world, scene, image, sort):
    monkeypatch.setenv("RTAMD_MULTI_LOOPBACK", "1")
    osc, psc = _scenes(scene, image)
    m = R.MultiRenderer(psc, [0] * world, sort=sort, L=R.test_lib())
    try:
        assert m.ranks == world
        P = psc.passes
        for n in (P, 3, 1, 0, -1):         # 1 and 0: fewer passes than devices, an idle rank
            st = m.run(n)
            k = P if n < 0 else n
            ref, ost = osc.render(sort=sort, pass_begin=0, pass_count=k)
            assert np.array_equal(m.framebuffer(), ref), (n, world)
            assert st["passes"] == k and st["live_segments"] == ost["live_segments"]
    finally:
        m.close()


def test_multi_renderer_refuses_missing_devices():
    _, psc = _scenes("cornell", (16, 16, 20, 2))
    with pytest.raises(R.RtError, match="no such HIP device"):
        R.MultiRenderer(psc, [0, R.device_count()])
    with pytest.raises(R.RtError, match="twice"):
        R.MultiRenderer(psc, [0, 0])


def test_bench_gpus2_without_torchrun_loopback(tmp_path):
    """`python bench.py --gpus 2` with WORLD_SIZE unset runs the in-library backend (rt_multi over GPUs 0..1); on
    this box through the test build's loopback transport.  The line says n_gpus 2 and n_ranks_seen 2, and the timed
    cornell_plus frame (BASELINE config 2, whole frame) equals the oracle's frame hash (tests/golden/
    bench_frames.json)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(RTAMD_LIB=R.TEST_LIB_PATH, RTAMD_MULTI_LOOPBACK="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--scene", "cornell_plus",
                        "--warmup", "1", "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps({k: line[k] for k in ("value", "ms_per_step", "n_gpus", "steps")}))
    assert line["n_gpus"] == 2 and line["config"]["n_ranks_seen"] == 2
    assert "rt_multi" in line["config"]["launch"] and "loopback" in line["config"]["launch"]
    assert line["parity"]["frame_bit_exact_vs_oracle"] is True
    assert line["bit_exact_vs_oracle"] is True


def test_bench_inlib_one_gpu_rccl():
    """`bench.py --inlib` at N = 1: the product library's rt_multi over a one-device RCCL communicator (the path
    `--gpus N` takes without torchrun); the timed cornell_plus frame equals the oracle's frame hash."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "RTAMD_LIB")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--inlib", "--scene", "cornell_plus",
                        "--warmup", "1", "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["config"]["n_ranks_seen"] == 1 and "rt_multi" in line["config"]["launch"]
    assert line["parity"]["frame_bit_exact_vs_oracle"] is True and line["bit_exact_vs_oracle"] is True
