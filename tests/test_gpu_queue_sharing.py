"""The pass scheduler's cross-stream waits on few hardware queues (round 5; DESIGN §9, the CU-mask hang).

HIP maps the renderer's streams -- one per pass in flight -- onto GPU_MAX_HW_QUEUES hardware queues (4 by
default), so with 20 passes in flight five streams share each in-order queue, and a stream's wait for another
stream's event blocks every packet behind it in that queue.  The scheduler only ever waits for an event that
the same host thread recorded earlier (a context's stream waits for the previous pass's framebuffer add, the
run's start event, and the final join), so the earliest unfinished packet in enqueue order never waits for a
later one and every sharing of queues makes progress.  This renders 25 passes with 20 in flight, staggered
starts (the delay kernels occupy their queue) and the synchronous and overlapped (run_async / wait_pass)
forms on 2 hardware queues, in a child process under a time limit, bit-exact against the oracle."""
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
IMAGE = (96, 64, 500, 8)            # 25 passes of 20 spp

CHILD = r"""
import hashlib, json, os, sys
sys.path[:0] = [os.path.join(%(repo)r, "cuda-raytracer_amd")]
import numpy as np, torch
torch.cuda.set_device(0)            # torch's HIP runtime first, as in the other torch + librtamd tests
import rtamd as R
psc = R.Scene(os.path.join(R.ASSETS, "cornell_plus.scene"), image=%(image)r)
out = {}
fb, st = R.render(psc, sort=True)
out["render"] = hashlib.sha256(np.asarray(fb, dtype="<f4").tobytes()).hexdigest()
ren = R.Renderer(psc, sort=True)
sums = torch.zeros((psc.passes, psc.pixels * 3), dtype=torch.float32, device="cuda")
side = torch.cuda.Stream()
ren.run_async(0, psc.passes, 1, sums.data_ptr())
acc = torch.zeros(psc.pixels * 3, dtype=torch.float32, device="cuda")
for k in range(psc.passes):                 # a caller stream waiting pass by pass, as the exchange does
    ren.wait_pass(k, side.cuda_stream)
    with torch.cuda.stream(side):
        acc += sums[k]
ren.finish()
side.synchronize()
out["async_fb"] = hashlib.sha256(np.asarray(ren.framebuffer(), dtype="<f4").tobytes()).hexdigest()
out["async_sum"] = hashlib.sha256(acc.cpu().numpy().astype("<f4").tobytes()).hexdigest()
ren.close()
print(json.dumps(out))
"""


def test_twenty_streams_on_two_queues_bitexact():
    if R.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    osc = O.OracleScene("%s/cornell_plus.scene" % R.ASSETS, image=IMAGE)
    ofb, _ = osc.render(sort=True)
    want = hashlib.sha256(np.asarray(ofb, dtype="<f4").tobytes()).hexdigest()
    env = dict(os.environ, GPU_MAX_HW_QUEUES="2", RTAMD_INFLIGHT="20", RTAMD_STAGGER_US="300")
    res = subprocess.run([sys.executable, "-c", CHILD % {"repo": REPO, "image": IMAGE}], env=env, cwd=REPO,
                         capture_output=True, text=True, timeout=150)
    assert res.returncode == 0, res.stderr[-3000:]
    got = json.loads(res.stdout.strip().splitlines()[-1])
    assert got["render"] == want
    assert got["async_fb"] == want
    # the caller's own pass-by-pass sum is (((0 + s0) + s1) + ...), the renderer's order
    assert got["async_sum"] == want
