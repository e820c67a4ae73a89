"""rt_renderer_run_async / rt_renderer_wait_pass / rt_renderer_finish (the overlapped multi-GPU exchange's
renderer side) through the C ABI: a caller's stream that waits for pass k reads pass k's finished sums while
the renderer may still render later passes; the run's framebuffer, pass sums and counters equal rt_renderer_run's
and the oracle's bit for bit (the reference's pass loop, raytracing.cu:222-254)."""
import numpy as np
import pytest

import oracle_lib as O
import rtamd as R

pytestmark = pytest.mark.gpu

IMAGE = (96, 54, 60, 16)           # 3 passes


@pytest.fixture(scope="module")
def torch_gpu():
    import torch
    if R.device_count() < 1 or not torch.cuda.is_available():
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    torch.cuda.set_device(0)
    return torch


@pytest.mark.parametrize("sort", [True, False])
def test_async_run_bitexact(torch_gpu, sort):
    torch = torch_gpu
    path = "%s/teapot.scene" % R.ASSETS
    osc, psc = O.OracleScene(path, image=IMAGE), R.Scene(path, image=IMAGE)
    ref_sums = osc.pass_sums(sort=sort, pass_begin=0, pass_count=psc.passes)
    ref_fb, ref_st = osc.render(sort=sort)
    ren = R.Renderer(psc, sort=sort)
    try:
        out = torch.zeros((psc.passes, psc.pixels * 3), dtype=torch.float32, device="cuda")
        side = torch.cuda.Stream()
        copies = []
        ren.run_async(0, psc.passes, 1, out.data_ptr())
        for k in range(psc.passes):             # each copy is ordered after its own pass only
            ren.wait_pass(k, side.cuda_stream)
            with torch.cuda.stream(side):
                copies.append(out[k].clone())
        st = ren.finish()
        side.synchronize()
        for k in range(psc.passes):
            assert np.array_equal(copies[k].cpu().numpy(), ref_sums[k]), "pass %d" % k
        assert np.array_equal(ren.framebuffer(), ref_fb)
        assert st["live_segments"] == ref_st["live_segments"] and st["passes"] == psc.passes
    finally:
        ren.close()


def test_async_run_misuse_is_refused(torch_gpu):
    torch = torch_gpu
    path = "%s/cornell.scene" % R.ASSETS
    psc = R.Scene(path, image=(32, 32, 40, 4))
    ren = R.Renderer(psc, sort=True)
    try:
        out = torch.zeros((2, psc.pixels * 3), dtype=torch.float32, device="cuda")
        with pytest.raises(R.RtError):
            ren.run_async(0, 2, 1, None)                    # the pass sums buffer is required
        with pytest.raises(R.RtError):
            ren.finish()                                    # nothing in flight
        ren.set_event_timing(False)
        ren.run_async(0, 2, 1, out.data_ptr())
        with pytest.raises(R.RtError):
            ren.run_async(0, 2, 1, out.data_ptr())          # the previous run is not finished
        with pytest.raises(R.RtError):
            ren.wait_pass(2, torch.cuda.current_stream().cuda_stream)   # no pass 2 in this run
        # every call that would run passes, touch the framebuffer or change the pending run's
        # settings is refused until finish() (finish used to read the current settings)
        dev = torch.zeros(psc.pixels * 3, dtype=torch.float32, device="cuda")
        for call in (lambda: ren.run(0, 1), lambda: ren.run_host(0, 1), ren.clear, ren.framebuffer,
                     lambda: ren.copy_framebuffer(dev.data_ptr()), lambda: ren.set_event_timing(True),
                     lambda: ren.set_counters(True), lambda: ren.launch_profile()):
            with pytest.raises(R.RtError):
                call()
        st = ren.finish()                                   # the run's stats, with the run's (off) timing
        assert st["passes"] == 2 and st["process_ms"] == 0.0
        fb_async = ren.framebuffer()
        np.testing.assert_array_equal(fb_async, out.sum(0).cpu().numpy())   # fb += pass sums, in order
        ren.set_event_timing(True)
        with pytest.raises(R.RtError):
            ren.wait_pass(0, torch.cuda.current_stream().cuda_stream)   # the run is finished
        ren.run(0, 2)                                       # the renderer is usable again
    finally:
        ren.close()


def test_accumulate_off_writes_pass_sums_only(torch_gpu):
    """rt_renderer_set_accumulate(0) (round 5, the multi-GPU drivers): the run writes each pass's sums, bit-exact
    against the oracle's, and adds nothing into the renderer's framebuffer; without a pass sums buffer such a
    run is refused."""
    torch = torch_gpu
    path = "%s/teapot.scene" % R.ASSETS
    osc, psc = O.OracleScene(path, image=IMAGE), R.Scene(path, image=IMAGE)
    ref_sums = osc.pass_sums(sort=True, pass_begin=0, pass_count=psc.passes)
    ren = R.Renderer(psc, sort=True)
    try:
        ren.set_accumulate(False)
        with pytest.raises(R.RtError):
            ren.run(0, 1)                                   # nowhere to put the sums
        out = torch.zeros((psc.passes, psc.pixels * 3), dtype=torch.float32, device="cuda")
        ren.run(0, psc.passes, 1, out.data_ptr())
        for k in range(psc.passes):
            assert np.array_equal(out[k].cpu().numpy(), ref_sums[k]), "pass %d" % k
        out.zero_()
        ren.run_async(0, psc.passes, 1, out.data_ptr())
        with pytest.raises(R.RtError):
            ren.set_accumulate(True)                        # refused while the run is pending
        ren.finish()
        for k in range(psc.passes):
            assert np.array_equal(out[k].cpu().numpy(), ref_sums[k]), "async pass %d" % k
        assert not ren.framebuffer().any()                  # nothing was accumulated
        ren.set_accumulate(True)
        ren.run(0, psc.passes)
        ref_fb, _ = osc.render(sort=True)
        assert np.array_equal(ren.framebuffer(), ref_fb)
    finally:
        ren.close()
