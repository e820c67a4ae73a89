"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the same inputs.

The contract is bit-exact: same seeds, same per-ray arithmetic (no FMA contraction, IEEE
div/sqrt, the same sin/cos/atan kernels), same traversal order, the same stable reorder and
the same per-pixel summation order.  Traversal work counters must match the oracle's
instrumented reference-order traversal exactly as well.
"""
import numpy as np
import pytest

import oracle_lib as O
import rtamd as R

pytestmark = pytest.mark.gpu

CASES = [
    # scene, image (W, H, spp, bounces), sort, use_bvh
    ("cornell", (64, 64, 24, 4), False, True),
    ("cornell", (64, 64, 24, 4), True, True),
    ("cornell_plus", (48, 48, 20, 8), True, True),
    ("cornell_plus", (48, 48, 20, 8), False, False),
    ("spheres", (64, 48, 20, 8), True, True),
    ("teapot", (96, 54, 20, 16), True, True),
    ("teapot", (96, 54, 20, 16), False, True),
    ("glass_teapot", (96, 54, 20, 16), True, True),
    ("lamp_available", (80, 45, 20, 32), True, True),
    ("cornell", (16, 16, 3, 0), True, True),          # zero bounces: black image
    ("spheres", (33, 17, 7, 1), False, True),         # odd sizes, one bounce, partial pass
]


def _pair(scene, image, use_bvh=True):
    path = "%s/%s.scene" % (R.ASSETS, scene)
    return O.OracleScene(path, use_bvh=use_bvh, image=image), R.Scene(path, use_bvh=use_bvh, image=image)


@pytest.fixture(scope="module")
def gpu():
    if R.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    return 0


def _diff(a, b):
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    return "max %.3g, rms %.3g, %d/%d differ" % (d.max(), np.sqrt((d * d).mean()), int((d > 0).sum()), d.size)


@pytest.mark.parametrize("scene,image,sort,use_bvh", CASES)
def test_render_bitexact(gpu, scene, image, sort, use_bvh):
    osc, psc = _pair(scene, image, use_bvh)
    ofb, ost = osc.render(sort=sort)
    gfb, gst = R.render(psc, sort=sort, counters=True)
    assert gfb.shape == ofb.shape
    assert np.array_equal(gfb, ofb), _diff(gfb, ofb)
    assert gst["live_segments"] == ost["live_segments"]
    assert gst["nodes_popped"] == ost["nodes_popped"]
    assert gst["internal_visits"] == ost["internal_visits"]
    assert gst["triangle_tests"] == ost["triangle_tests"]
    assert gst["misses"] == ost["misses"]
    assert gst["hits"] == ost["hits_triangle"] + ost["hits_sphere"]
    assert gst["generated_rays"] == image[0] * image[1] * image[2]


def test_pass_sharding_matches_full_render(gpu):
    """Passes rendered in two strided halves (the multi-GPU pass shard) sum to the same image."""
    image = (64, 64, 60, 6)
    _, psc = _pair("cornell_plus", image)
    full, _ = R.render(psc, sort=True)
    r0 = R.Renderer(psc, sort=True)
    sums = []
    for p in range(psc.passes):
        r0.clear()
        r0.run(pass_begin=p, count=1)
        sums.append(r0.framebuffer())
    acc = np.zeros_like(full)
    for s in sums:
        acc = acc + s
    assert np.array_equal(acc, full)
    r0.clear()
    r0.run(pass_begin=1, count=-1, stride=2)
    odd = r0.framebuffer()
    assert np.array_equal(odd, (np.zeros_like(full) + sums[1]))


def test_device_warmup(gpu):
    R.warmup(0)
    R.warmup(0)                       # idempotent
    with pytest.raises(R.RtError):
        R.warmup(R.device_count())    # no such device


def test_bloom_bitexact(gpu):
    rng = np.random.default_rng(7)
    w, h = 97, 61
    fb = (rng.random(w * h * 3, dtype=np.float32) * 40).astype(np.float32)
    thr = np.float32(0.7 * 20)
    assert np.array_equal(R.bloom(fb, w, h, thr, 5), O.bloom(fb, w, h, thr, 5))


def test_cli_gpu_png_matches_oracle(gpu, tmp_path):
    """`raytracing <scene> --image ...` end to end: GPU render, GPU bloom, tone map, PNG."""
    import subprocess
    from test_cpu_path import _decode_png
    image = (64, 48, 40, 6)
    r = subprocess.run([R.CLI_PATH, "cornell_plus.scene", "--image", *map(str, image), "1", "--out",
                        str(tmp_path / "o.png")], cwd=R.ASSETS, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "GPU Took" in r.stdout
    sc = O.OracleScene("%s/cornell_plus.scene" % R.ASSETS, image=image)
    fb, _ = sc.render(sort=True)
    fb = O.bloom(fb, 64, 48, np.float32(0.7 * 40), 5)
    want = O.tonemap(fb, 64, 48, 1.0, 40).reshape(48, 64, 3)
    assert np.array_equal(_decode_png(str(tmp_path / "o.png")), want)


def test_cli_multi_device_equals_single(gpu, tmp_path):
    """--devices N (the in-library RCCL pass sharding, rt_opts.device_count) gives the 1-device
    image; with one GPU on the box N=1 is the only runnable case: the RCCL communicator, the
    slice all-to-all, the owner's ordered adds and the gather all run with one rank."""
    import subprocess
    args = ["cornell.scene", "--image", "48", "48", "60", "4", "1"]
    a = subprocess.run([R.CLI_PATH] + args + ["--out", str(tmp_path / "a.png")], cwd=R.ASSETS, capture_output=True)
    b = subprocess.run([R.CLI_PATH] + args + ["--devices", "1", "--out", str(tmp_path / "b.png")], cwd=R.ASSETS,
                       capture_output=True)
    assert a.returncode == 0 and b.returncode == 0
    assert open(tmp_path / "a.png", "rb").read() == open(tmp_path / "b.png", "rb").read()


def test_many_passes_in_flight_bitexact(gpu):
    """10 passes (4 in flight on separate streams): the ordered framebuffer adds must reproduce
    the oracle's pass-ordered sum exactly, for sort on and off."""
    image = (40, 32, 190, 5)                     # 10 passes, the last one 10 spp
    for sort in (True, False):
        osc, psc = _pair("cornell_plus", image)
        ofb, ost = osc.render(sort=sort)
        gfb, gst = R.render(psc, sort=sort)
        assert np.array_equal(gfb, ofb), _diff(gfb, ofb)
        assert gst["live_segments"] == ost["live_segments"]


def test_run_host_pass_sums(gpu):
    image = (32, 32, 100, 4)
    osc, psc = _pair("cornell", image)
    want = osc.pass_sums(sort=True, pass_begin=1, pass_count=2)
    r = R.Renderer(psc, sort=True)
    sums, st = r.run_host(pass_begin=1, count=2, stride=2)      # passes 1 and 3
    assert np.array_equal(sums[0], want[0])
    assert np.array_equal(sums[1], osc.pass_sums(sort=True, pass_begin=3, pass_count=1)[0])
    r.close()


@pytest.mark.parametrize("fused", ["0", "1", "2", "3"])   # never, every bounce, bounce 0, bounces 0-1
@pytest.mark.parametrize("scene,image,sort", [("teapot", (96, 54, 20, 16), True), ("cornell_plus", (48, 48, 20, 8), False),
                                              ("spheres", (64, 48, 20, 8), True)])
def test_fused_and_plain_reorder_bitexact(gpu, monkeypatch, scene, image, sort, fused):
    # both reorder variants (shade writes the state and the scatter moves it, or the scatter replays
    # the shading; the renderer picks by scene size, RTAMD_FUSED forces one) against the oracle
    monkeypatch.setenv("RTAMD_FUSED", fused)
    osc, psc = _pair(scene, image)
    ofb, ost = osc.render(sort=sort)
    gfb, gst = R.render(psc, sort=sort, counters=True)
    assert np.array_equal(gfb, ofb), _diff(gfb, ofb)
    assert gst["live_segments"] == ost["live_segments"]
    assert gst["hits"] == ost["hits_triangle"] + ost["hits_sphere"] and gst["misses"] == ost["misses"]


@pytest.mark.parametrize("home", ["0", "1"])
@pytest.mark.parametrize("scene,image", [("teapot", (96, 54, 40, 16)), ("cornell_plus", (48, 40, 60, 8)),
                                         ("spheres", (64, 48, 40, 8))])
def test_home_indexed_radiance_bitexact(gpu, monkeypatch, scene, image, home):
    """Sort on with the fused bounce-0 reorder (round 5): a surviving ray's radiance lives at its home index (its
    bounce-1 slot), the replay writes bounce-0 emission there and home_of[ray id] for the accumulation; RTAMD_HOME=0
    keeps acc[ray id].  cornell_plus has an emitter (radiance terms at bounce 0 and later, the read-modify-write
    path), spheres runs the fused replay at every bounce; both forms equal the oracle bit for bit."""
    monkeypatch.setenv("RTAMD_HOME", home)
    osc, psc = _pair(scene, image)
    ofb, ost = osc.render(sort=True)
    gfb, gst = R.render(psc, sort=True)
    assert np.array_equal(gfb, ofb), _diff(gfb, ofb)
    assert gst["live_segments"] == ost["live_segments"]


@pytest.mark.parametrize("scene,image,sort", [("cornell_plus", (40, 32, 350, 5), True),    # 18 passes: two calls of 16
                                              ("cornell", (33, 17, 190, 4), False),        # 10 passes, odd size
                                              ("teapot", (64, 36, 45, 16), True)])         # short last pass
@pytest.mark.parametrize("xchg", ["overlap", "overlap-rccl", "overlap1", "sync"])
def test_multi_device_rccl_bitexact(gpu, monkeypatch, scene, image, sort, xchg):
    """rt_render with rt_opts.device_count (in-library pass sharding over an RCCL communicator,
    slice all-to-all, ordered owner adds, gather to the first device) at N = 1, the only device
    count this box has: bit-exact against the oracle and the single-device render.  The exchange
    runs overlapped with the render (round 5: every 4 rounds, or every round) or after each chunk.
    At N = 1 the all-to-all and the gather are the identity and are skipped; "overlap-rccl", "overlap1" and
    "sync" run them through RCCL anyway (RTAMD_XCHG_IDENTITY=0)."""
    if xchg != "overlap":
        monkeypatch.setenv("RTAMD_XCHG_IDENTITY", "0")
    monkeypatch.setenv("RTAMD_XCHG_CHUNK", "16")            # more than 16 rounds: two renderer calls
    if xchg == "sync":
        monkeypatch.setenv("RTAMD_XCHG_OVERLAP", "0")
    elif xchg == "overlap1":
        monkeypatch.setenv("RTAMD_XCHG_ROUNDS", "1")
    osc, psc = _pair(scene, image)
    ofb, ost = osc.render(sort=sort)
    gfb, gst = R.render(psc, sort=sort, devices=[0])
    assert np.array_equal(gfb, ofb), _diff(gfb, ofb)
    assert gst["live_segments"] == ost["live_segments"]
    assert gst["passes"] == psc.passes
    assert gst["exchange_ms"] > 0


@pytest.mark.parametrize("world,scene,image,sort,xchg", [
    (2, "teapot", (64, 36, 100, 16), True, "overlap"),       # 5 passes: device 1 has no pass in the last round
    (3, "cornell_plus", (40, 32, 350, 5), True, "overlap1"),  # 18 passes, 6 rounds
    (5, "cornell", (33, 17, 190, 4), False, "sync"),          # 10 passes, odd size: padded slices
    (2, "cornell", (24, 16, 700, 3), True, "overlap"),        # 35 passes = 18 rounds: two calls of 16 rounds
    (2, "cornell", (24, 16, 700, 3), True, "overlap-1call"),  # the same in one call (the default chunk)
])
def test_multi_device_loopback_bitexact(gpu, monkeypatch, world, scene, image, sort, xchg):
    """The in-library multi-device render at N > 1 on the box's one GPU (round 5): RTAMD_MULTI_LOOPBACK=1 runs
    rt_multi.hip's device threads on the same GPU with its two collectives as device-to-device copies (RCCL refuses
    two ranks on one GPU), so the pass dealing, the stale rows of rounds a device has no pass in, the overlapped
    exchange, the owners' ordered adds and the gather all run at N = 2 / 3 / 5: bit-exact against the oracle."""
    monkeypatch.setenv("RTAMD_MULTI_LOOPBACK", "1")   # read by the test build only (librtamd_test.so)
    if xchg != "overlap-1call":
        monkeypatch.setenv("RTAMD_XCHG_CHUNK", "16")
    if xchg == "sync":
        monkeypatch.setenv("RTAMD_XCHG_OVERLAP", "0")
    elif xchg == "overlap1":
        monkeypatch.setenv("RTAMD_XCHG_ROUNDS", "1")
    osc, psc = _pair(scene, image)
    ofb, ost = osc.render(sort=sort)
    T = R.test_lib()
    gfb, gst = R.render(psc, sort=sort, devices=[0] * world, L=T)
    assert np.array_equal(gfb, ofb), _diff(gfb, ofb)
    assert gst["live_segments"] == ost["live_segments"] and gst["passes"] == psc.passes
    with pytest.raises(R.RtError, match="pass sharding only"):
        R.render(psc, sort=sort, devices=[0] * world, shard_tiles=True, L=T)
    # the product library has no loopback transport: the same device list is refused
    with pytest.raises(R.RtError, match="twice"):
        R.render(psc, sort=sort, devices=[0] * world)


def test_multi_device_rejects_bad_device_lists(gpu):
    _, psc = _pair("cornell", (16, 16, 20, 2))
    with pytest.raises(R.RtError, match="twice"):
        R.render(psc, devices=[0, 0])
    with pytest.raises(R.RtError, match="no such"):
        R.render(psc, devices=[0, R.device_count()])
    with pytest.raises(R.RtError, match="whole frame"):
        R.render(psc, devices=[0], pass_begin=1)


@pytest.mark.parametrize("sort", [True, False])
def test_renderer_reuse_bitexact(gpu, sort):
    """A renderer reused across runs -- first the short remainder pass (5 rays per pixel), then the whole
    frame twice -- renders the frame exactly as the oracle does each time (no state carried between
    runs: live counts, trace queues, reorder counts and per-pass buffers are reset per pass)."""
    image = (96, 54, 45, 16)
    osc, psc = _pair("teapot", image)
    ofb, _ = osc.render(sort=sort)
    r = R.Renderer(psc, sort=sort)
    r.run(pass_begin=2, count=1)
    for _ in range(2):
        r.clear()
        r.run(pass_begin=0, count=-1)
        fb = r.framebuffer()
        assert np.array_equal(fb, ofb), _diff(fb, ofb)
