"""The multi-device abort protocol of the in-library multi-GPU render (csrc/rt_multi.hip over RCCL),
exercised on the CPU: csrc/mgpu_protocol.h is the same code the library runs, driven here by device
threads with fake communicators (tests/native/mgpu_protocol_test.cpp).  A device failing after the
setup barrier while its peers sit in a collective that can never complete must release every peer
(each aborts its own communicator) -- the path a one-GPU box cannot reach (world 1 installs no
exchange).  Reference: the reference renders on one device (raytracing.cu:170-284); this guards the
multi-device extension only."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.fixture(scope="module", params=["plain", "tsan"])
def prog(request, tmp_path_factory):
    """The test program, plain and under ThreadSanitizer (host code only: the protocol is CPU code)."""
    out = str(tmp_path_factory.mktemp("mgpu") / ("mgpu_protocol_test_" + request.param))
    flags = ["-fsanitize=thread", "-g"] if request.param == "tsan" else []
    subprocess.run(["g++", "-std=c++17", "-O1", "-pthread", "-Wall", "-Werror"] + flags +
                   ["-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "cuda-raytracer_amd", "csrc"),
                    os.path.join(HERE, "native", "mgpu_protocol_test.cpp"), "-o", out], check=True)
    return out


def run(prog, *args):
    p = subprocess.run([prog] + [str(a) for a in args], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "ThreadSanitizer" not in p.stderr, p.stderr
    words = p.stdout.split()
    i = words.index("aborted")
    return [int(x) for x in words[1:i]], int(words[i + 1]), int(words[i + 3]), int(words[i + 5])


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_all_devices_complete(prog, world):
    rc, aborted, failed, entered = run(prog, world, "ok")
    assert rc == [0] * world and aborted == 0 and failed == 0 and entered == 3 * world


@pytest.mark.parametrize("world,rank", [(2, 0), (2, 1), (4, 3), (8, 5)])
def test_setup_failure_returns_before_any_collective(prog, world, rank):
    rc, aborted, failed, entered = run(prog, world, "setup", rank)
    assert rc[rank] == -5                                 # RT_E_OOM, the device's own error
    assert all(r == -1 for i, r in enumerate(rc) if i != rank)  # RT_E_INVALID: a peer failed
    assert entered == 0                                  # nobody entered a collective
    assert aborted == world - 1 and failed == 1          # the others drop their unused communicators


@pytest.mark.parametrize("world,rank", [(2, 0), (2, 1), (4, 2), (8, 7)])
def test_failure_after_setup_releases_blocked_peers(prog, world, rank):
    for _ in range(5):                                   # thread interleavings vary run to run
        rc, aborted, failed, _ = run(prog, world, "after", rank)
        assert rc[rank] != 0 and all(r != 0 for r in rc)  # nobody reports success, nobody hangs
        assert aborted == world and failed == 1          # every device aborted its own communicator
