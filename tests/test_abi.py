"""The C ABI boundary (include/rt_abi.h): library loads, exports every declared symbol, and the
ctypes mirror matches the C struct layouts.  No HIP compute calls (runs without a GPU)."""
import ctypes as C
import re
import subprocess

import rtamd as R


def declared_functions():
    text = open(R.HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_drop_in_entry_points():
    names = declared_functions()
    for n in ("rt_render", "rt_scene_load", "rt_bloom", "rt_tonemap", "rt_write_png", "rt_cpu_render",
              "rt_renderer_create", "rt_renderer_run", "rt_last_error"):
        assert n in names


def test_library_exports_every_declared_symbol():
    lib = R.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", R.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines())
    assert set(declared_functions()) <= exported


def test_library_is_gfx950_and_links_hip():
    blob = open(R.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}
    ldd = subprocess.run(["ldd", R.LIB_PATH], capture_output=True, text=True).stdout
    assert "libamdhip64" in ldd


def test_struct_layouts():
    # sizes fixed by the reference layouts (scene.cuh:9-100) and by rt_abi.h
    assert C.sizeof(R.RtScene) == 216
    assert C.sizeof(R.RtOpts) == 56   # + tile_count/index/rows, device_count, device_ids*, shard_tiles
    assert C.sizeof(R.RtLoadOpts) == 48
    assert C.sizeof(R.RtStats) == 11 * 8 + 8 + 5 * 8 + 8 + 8
    assert R.lib().rt_abi_version() == 7


def test_default_options():
    o = R.RtOpts()
    R.lib().rt_default_opts(C.byref(o))
    assert (o.sort, o.device, o.pass_begin, o.pass_count, o.pass_stride, o.collect_counters) == (1, 0, 0, -1, 1, 0)
    assert (o.tile_count, o.tile_index, o.tile_rows) == (0, 0, 0)   # whole image, 8-row stripes
    assert o.device_count == 0 and not o.device_ids and o.shard_tiles == 0   # one device, no RCCL


def test_tile_rows_of():
    # 8-row stripes dealt round-robin; the image's last stripe may be short
    assert R.tile_rows_of(20, 2, 0) == list(range(0, 8)) + list(range(16, 20))
    assert R.tile_rows_of(20, 2, 1) == list(range(8, 16))
    assert R.tile_rows_of(20, 4, 3) == []
    for h, t, r in ((1080, 8, 8), (37, 3, 5), (9, 5, 2)):
        rows = sorted(x for i in range(t) for x in R.tile_rows_of(h, t, i, r))
        assert rows == list(range(h))


def test_invalid_arguments_fail_loudly():
    lib = R.lib()
    assert lib.rt_render(None, None, None, None) < 0
    assert b"null" in lib.rt_last_error()
    assert lib.rt_renderer_run(None, 0, 1, 1, None, None) < 0
    assert lib.rt_write_png(b"/nonexistent/x.png", None, 1, 1) < 0


def test_test_hooks_only_in_the_test_build():
    """The one-GPU loopback transport and the failure injection are compiled into librtamd_test.so only
    (-DRTAMD_TEST_HOOKS): no environment variable can switch the product library's collectives."""
    for var in (b"RTAMD_MULTI_LOOPBACK", b"RTAMD_FAIL_AFTER_SETUP"):
        assert var not in open(R.LIB_PATH, "rb").read()
        assert var in open(R.TEST_LIB_PATH, "rb").read()
    assert R.test_lib().rt_abi_version() == R.lib().rt_abi_version()


def test_library_sets_the_hardware_queue_default():
    """Loading librtamd.so asks HIP for 24 hardware queues unless the host set GPU_MAX_HW_QUEUES (a
    constructor that runs before the host's first HIP call), and keeps a host's own value."""
    code = ("import ctypes, sys; ctypes.CDLL(sys.argv[1]); libc = ctypes.CDLL(None); "
            "libc.getenv.restype = ctypes.c_char_p; print(libc.getenv(b'GPU_MAX_HW_QUEUES').decode())")
    env = {k: v for k, v in __import__("os").environ.items() if k != "GPU_MAX_HW_QUEUES"}
    out = subprocess.run([__import__("sys").executable, "-c", code, R.LIB_PATH], env=env, capture_output=True,
                         text=True, check=True).stdout.split()
    assert out == ["24"]
    env["GPU_MAX_HW_QUEUES"] = "6"
    out = subprocess.run([__import__("sys").executable, "-c", code, R.LIB_PATH], env=env, capture_output=True,
                         text=True, check=True).stdout.split()
    assert out == ["6"]
