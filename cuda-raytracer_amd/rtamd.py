"""ctypes host binding of librtamd.so (include/rt_abi.h) for Python callers.

This is plumbing for tests, the benchmark and the multi-GPU driver: every render call goes
through the C ABI into the HIP kernels.  There is no Python or CPU fallback for the GPU
path: if the library or a HIP device is missing, the calls raise.
"""
import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
BUILD_DIR = os.path.join(PKG_DIR, "build")
# Up to 20 passes in flight on their own streams: HIP needs a hardware queue per stream.  Loading
# librtamd.so asks for 24 unless the variable is set (rt_abi.h); setting the same default here also
# covers a process where torch initialises HIP before the library loads.  A caller's value stands.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "24")
LIB_PATH = os.environ.get("RTAMD_LIB") or os.path.join(BUILD_DIR, "librtamd.so")  # env: A/B builds only
# the same library with the multi-GPU test hooks (one-GPU loopback transport, failure injection):
# tests only, loaded beside the product library (test_lib())
TEST_LIB_PATH = os.path.join(BUILD_DIR, "librtamd_test.so")
CLI_PATH = os.path.join(BUILD_DIR, "raytracing")
HEADER = os.path.join(REPO, "include", "rt_abi.h")
ASSETS = os.path.join(REPO, "assets")


class RtError(RuntimeError):
    pass


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


P = C.c_void_p
I32 = C.c_int32


class RtScene(C.Structure):
    _fields_ = [("spheres", P), ("sphere_count", I32), ("triangles", P), ("triangle_count", I32),
                ("material_indices", P), ("materials", P), ("material_count", I32),
                ("bvh", P), ("bvh_node_count", I32), ("width", I32), ("height", I32),
                ("environment_map", P), ("environment_map_width", I32), ("environment_map_height", I32),
                ("camera_position", Vec3), ("forward", Vec3), ("up", Vec3),
                ("vertical_fov", C.c_float), ("exposure", C.c_float),
                ("min_coord", Vec3), ("inv_dimensions", Vec3),
                ("scaled_right", Vec3), ("scaled_up", Vec3), ("near_plane_top_left", Vec3),
                ("inv_width", C.c_float), ("inv_height", C.c_float),
                ("bounces", I32), ("ray_count", I32)]


class RtLoadOpts(C.Structure):
    _fields_ = [("use_bvh", I32), ("quiet", I32), ("asset_root", C.c_char_p), ("image_override", I32),
                ("width", I32), ("height", I32), ("ray_count", I32), ("bounces", I32),
                ("exposure_override", I32), ("exposure", C.c_float), ("bvh_device", I32)]


class RtOpts(C.Structure):
    _fields_ = [("sort", I32), ("device", I32), ("pass_begin", I32), ("pass_count", I32),
                ("pass_stride", I32), ("collect_counters", I32),
                ("tile_count", I32), ("tile_index", I32), ("tile_rows", I32),
                ("device_count", I32), ("device_ids", C.POINTER(I32)), ("shard_tiles", I32)]


# rt_exchange_fn: (user, bytes, n, hip_stream) -> 0 (pixel tiles with sort on, rt_renderer_set_exchange)
EXCHANGE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint8), C.c_uint64, C.c_void_p)


class RtStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("generated_rays", "live_segments", "sorted_items",
                                          "nodes_popped", "internal_visits", "triangle_tests",
                                          "sphere_tests", "hits", "misses", "hits_sphere",
                                          "dead_slots")] + \
               [("passes", C.c_uint32), ("reserved", C.c_uint32)] + \
               [(n, C.c_double) for n in ("render_ms", "kernel_ms", "process_ms", "sort_ms", "trace_ms")] + \
               [("trace_launches", C.c_uint64), ("exchange_ms", C.c_double)]

    def as_dict(self):
        return {n: (float(getattr(self, n)) if t is C.c_double else int(getattr(self, n)))
                for n, t in self._fields_ if n != "reserved"}


_lib = None


def build(jobs=8):
    subprocess.run(["make", "-s", "-j%d" % jobs, "-C", PKG_DIR], check=True)


_test_lib = None


def lib():
    """Load librtamd.so.  Raises if it has not been built: no fallback exists."""
    global _lib
    if _lib is None:
        _lib = _load(LIB_PATH)
    return _lib


def test_lib():
    """librtamd_test.so (the test-hook build: RTAMD_MULTI_LOOPBACK, RTAMD_FAIL_AFTER_SETUP), for tests.
    Scenes loaded through lib() can be passed to it: rt_scene is a plain host view."""
    global _test_lib
    if _test_lib is None:
        _test_lib = _load(TEST_LIB_PATH)
    return _test_lib


def _load(path):
    if not os.path.exists(path):
        raise RtError("%s is not built (run `make -C cuda-raytracer_amd` or "
                      "__graft_entry__.build())" % os.path.basename(path))
    L = C.CDLL(path)
    L.rt_last_error.restype = C.c_char_p
    L.rt_abi_version.restype = C.c_int
    L.rt_device_count.restype = C.c_int
    L.rt_default_opts.argtypes = [P]
    L.rt_default_load_opts.argtypes = [P]
    L.rt_scene_load.argtypes = [C.c_char_p, P, C.POINTER(P)]
    L.rt_scene_view.argtypes = [P]
    L.rt_scene_view.restype = C.POINTER(RtScene)
    L.rt_scene_bvh_ms.argtypes = [P]
    L.rt_scene_bvh_ms.restype = C.c_double
    L.rt_scene_free.argtypes = [P]
    L.rt_render.argtypes = [P, P, P, P]
    L.rt_renderer_create.argtypes = [P, P, C.POINTER(P)]
    L.rt_renderer_run.argtypes = [P, I32, I32, I32, P, P]
    L.rt_renderer_run_host.argtypes = [P, I32, I32, I32, P, P]
    L.rt_renderer_read_framebuffer.argtypes = [P, P]
    L.rt_renderer_clear.argtypes = [P]
    L.rt_renderer_set_counters.argtypes = [P, I32]
    L.rt_renderer_destroy.argtypes = [P]
    L.rt_trace_rays.argtypes = [P, P, P, I32, P, P, P]
    L.rt_bloom.argtypes = [P, I32, I32, C.c_float, I32, I32]
    L.rt_bloom_device.argtypes = [P, I32, I32, C.c_float, I32, I32]
    L.rt_tonemap.argtypes = [P, I32, I32, C.c_float, I32, P]
    L.rt_write_png.argtypes = [C.c_char_p, P, I32, I32]
    L.rt_cpu_render.argtypes = [P, P, I32, C.POINTER(C.c_double)]
    L.rt_multi_create.argtypes = [P, P, C.POINTER(P)]
    L.rt_multi_run.argtypes = [P, I32, P, P]
    L.rt_multi_read_framebuffer.argtypes = [P, P]
    L.rt_multi_set_event_timing.argtypes = [P, I32]
    L.rt_multi_set_counters.argtypes = [P, I32]
    L.rt_multi_ranks.argtypes = [P]
    L.rt_multi_destroy.argtypes = [P]
    return L


def _check(rc, L=None):
    if rc != 0:
        raise RtError("rt error %d: %s" % (rc, (L or lib()).rt_last_error().decode()))


def _ptr(a):
    return a.ctypes.data_as(P)


def warmup(device=0):
    """rt_device_warmup: HIP runtime, queues and code object initialised on `device`."""
    _check(lib().rt_device_warmup(device))


def device_count():
    return lib().rt_device_count()


class Scene:
    """A scene loaded by the product loader (rt_scene_load)."""

    def __init__(self, path, use_bvh=True, asset_root=ASSETS, image=None, exposure=None, quiet=True,
                 bvh_device=-1):
        """bvh_device >= 0 builds the BVH on that GPU (same arrays as the host build)."""
        L = lib()
        o = RtLoadOpts()
        L.rt_default_load_opts(C.byref(o))
        o.use_bvh = int(use_bvh)
        o.bvh_device = int(bvh_device)
        o.quiet = int(quiet)
        self._root = asset_root.encode() if asset_root else None
        o.asset_root = self._root
        if image is not None:
            o.image_override = 1
            o.width, o.height, o.ray_count, o.bounces = [int(v) for v in image]
        if exposure is not None:
            o.exposure_override = 1
            o.exposure = float(exposure)
        h = P()
        _check(L.rt_scene_load(path.encode(), C.byref(o), C.byref(h)))
        self.h = h
        self.view = L.rt_scene_view(h).contents

    def __del__(self):
        if getattr(self, "h", None):
            lib().rt_scene_free(self.h)
            self.h = None

    @property
    def ptr(self):
        return lib().rt_scene_view(self.h)

    @property
    def width(self):
        return self.view.width

    @property
    def height(self):
        return self.view.height

    @property
    def pixels(self):
        return self.view.width * self.view.height

    @property
    def passes(self):
        return (self.view.ray_count + 19) // 20

    @property
    def bvh_ms(self):
        return lib().rt_scene_bvh_ms(self.h)

    def arrays(self):
        v = self.view

        def arr(p, n, cols, dt=np.float32):
            if n == 0:
                return np.zeros((0, cols) if cols else 0, dt)
            itemsize = np.dtype(dt).itemsize * (cols or 1)
            buf = (C.c_char * (n * itemsize)).from_address(p)
            a = np.frombuffer(buf, dtype=dt).copy()
            return a.reshape(n, cols) if cols else a
        cam = np.array([v.camera_position.x, v.camera_position.y, v.camera_position.z,
                        v.forward.x, v.forward.y, v.forward.z, v.up.x, v.up.y, v.up.z,
                        v.vertical_fov] +
                       [c for vec in (v.min_coord, v.inv_dimensions, v.scaled_right, v.scaled_up,
                                      v.near_plane_top_left) for c in (vec.x, vec.y, vec.z)] +
                       [v.inv_width, v.inv_height, v.exposure, 0.0, 0.0], dtype=np.float32)
        return dict(spheres=arr(v.spheres, v.sphere_count, 4),
                    triangles=arr(v.triangles, v.triangle_count, 12),
                    material_indices=arr(v.material_indices, v.sphere_count + v.triangle_count, 0, np.uint16),
                    materials=arr(v.materials, v.material_count, 12),
                    bvh=arr(v.bvh, v.bvh_node_count, 8),
                    env=arr(v.environment_map, v.environment_map_width * v.environment_map_height, 3),
                    camera=cam)


def default_opts(sort=True, device=0, pass_begin=0, pass_count=-1, pass_stride=1, counters=False,
                 tiles=None):
    """tiles = (tile_count, tile_index[, tile_rows]): render only that owner's row stripes."""
    o = RtOpts()
    lib().rt_default_opts(C.byref(o))
    o.sort, o.device, o.pass_begin, o.pass_count = int(sort), device, pass_begin, pass_count
    o.pass_stride, o.collect_counters = pass_stride, int(counters)
    if tiles is not None:
        o.tile_count, o.tile_index = tiles[0], tiles[1]
        o.tile_rows = tiles[2] if len(tiles) > 2 else 0
    return o


def tile_rows_of(height, tile_count, tile_index, tile_rows=8):
    """Image rows owned by tile_index: stripes of tile_rows rows dealt round-robin (rt_opts)."""
    rows = []
    for k in range(tile_index, -(-height // tile_rows), tile_count):
        rows.extend(range(k * tile_rows, min((k + 1) * tile_rows, height)))
    return rows


def render(scene, sort=True, device=0, pass_begin=0, pass_count=-1, pass_stride=1, counters=False,
           tiles=None, devices=None, shard_tiles=False, L=None):
    """rt_render: the drop-in for gpu_raytrace.  Returns (framebuffer W*H*3 float32, stats).
    devices = list of device ordinals: the in-library multi-GPU render (pass sharding + RCCL
    slice exchange and gather; rt_opts.device_count/device_ids), also at one device.
    L = the library to call (default lib(); tests: test_lib())."""
    L = L or lib()
    fb = np.zeros(scene.pixels * 3, np.float32)
    st = RtStats()
    o = default_opts(sort, device, pass_begin, pass_count, pass_stride, counters, tiles)
    ids = None
    if devices is not None:
        ids = (I32 * len(devices))(*[int(d) for d in devices])
        o.device_count = len(devices)
        o.device_ids = C.cast(ids, C.POINTER(I32))
        o.shard_tiles = int(shard_tiles)
    _check(L.rt_render(scene.ptr, C.byref(o), _ptr(fb), C.byref(st)), L)
    return fb, st.as_dict()


class MultiRenderer:
    """rt_multi: the persistent in-library multi-GPU renderer (one process, one RCCL communicator over
    `devices`, pass sharding with the slice exchange; the frame is gathered on devices[0])."""

    def __init__(self, scene, devices, sort=True, counters=False, L=None):
        self.L = L or lib()
        self.scene = scene
        o = default_opts(sort, int(devices[0]) if devices else 0, counters=counters)
        self._ids = (I32 * len(devices))(*[int(d) for d in devices])
        o.device_count = len(devices)
        o.device_ids = C.cast(self._ids, C.POINTER(I32))
        h = P()
        _check(self.L.rt_multi_create(scene.ptr, C.byref(o), C.byref(h)), self.L)
        self.h = h
        self.devices = len(devices)

    def run(self, pass_count=-1, host=False):
        """Renders passes 0..pass_count-1 of the frame over the devices; returns stats (and the frame
        when host=True: (fb, stats))."""
        st = RtStats()
        fb = np.zeros(self.scene.pixels * 3, np.float32) if host else None
        _check(self.L.rt_multi_run(self.h, int(pass_count), _ptr(fb) if host else None, C.byref(st)), self.L)
        return (fb, st.as_dict()) if host else st.as_dict()

    def framebuffer(self):
        fb = np.zeros(self.scene.pixels * 3, np.float32)
        _check(self.L.rt_multi_read_framebuffer(self.h, _ptr(fb)), self.L)
        return fb

    @property
    def ranks(self):
        return self.L.rt_multi_ranks(self.h)

    def set_event_timing(self, on):
        _check(self.L.rt_multi_set_event_timing(self.h, int(on)), self.L)

    def set_counters(self, on):
        _check(self.L.rt_multi_set_counters(self.h, int(on)), self.L)

    def close(self):
        if getattr(self, "h", None):
            self.L.rt_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


RCCL_ID_BYTES = 128   # RT_RCCL_ID_BYTES


def rccl_unique_id():
    """rt_rccl_unique_id: a new RCCL communicator id (bytes) for set_exchange_rccl."""
    buf = (C.c_uint8 * RCCL_ID_BYTES)()
    f = lib().rt_rccl_unique_id
    f.argtypes = [P]
    _check(f(buf))
    return bytes(buf)


def trace_rays(scene, rays, device=0, counters=False):
    """rt_trace_rays: closest hit of rays (n, 6) float32 {o.xyz, d.xyz}.  Returns (t, index, stats)."""
    rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
    n = rays.shape[0]
    t = np.zeros(n, np.float32)
    idx = np.zeros(n, np.int32)
    st = RtStats()
    o = default_opts(True, device, counters=counters)
    _check(lib().rt_trace_rays(scene.ptr, C.byref(o), _ptr(rays), n, _ptr(t), _ptr(idx), C.byref(st)))
    return t, idx, st.as_dict()


class Renderer:
    """Persistent renderer (scene + ray buffers resident in HBM)."""

    def __init__(self, scene, sort=True, device=0, counters=False, tiles=None):
        self.scene = scene
        o = default_opts(sort, device, counters=counters, tiles=tiles)
        h = P()
        _check(lib().rt_renderer_create(scene.ptr, C.byref(o), C.byref(h)))
        self.h = h

    def run(self, pass_begin=0, count=1, stride=1, d_pass_sums=None):
        st = RtStats()
        _check(lib().rt_renderer_run(self.h, pass_begin, count, stride,
                                     P(d_pass_sums) if d_pass_sums else None, C.byref(st)))
        return st.as_dict()

    def run_async(self, pass_begin=0, count=1, stride=1, d_pass_sums=None):
        """rt_renderer_run_async: enqueue the passes and return; then wait_pass / finish."""
        f = lib().rt_renderer_run_async
        f.argtypes = [P, I32, I32, I32, P]
        _check(f(self.h, pass_begin, count, stride, P(d_pass_sums) if d_pass_sums else None))

    def wait_pass(self, k, hip_stream):
        """The HIP stream `hip_stream` (a raw handle, e.g. torch.cuda.current_stream().cuda_stream)
        waits until pass k of the async run has written its sums."""
        f = lib().rt_renderer_wait_pass
        f.argtypes = [P, I32, P]
        _check(f(self.h, int(k), P(hip_stream) if hip_stream else None))

    def finish(self):
        st = RtStats()
        f = lib().rt_renderer_finish
        f.argtypes = [P, P]
        _check(f(self.h, C.byref(st)))
        return st.as_dict()

    def run_host(self, pass_begin=0, count=1, stride=1):
        """Renders passes and returns their per-pass sums (count, W*H*3) in host memory."""
        out = np.zeros((count, self.scene.pixels * 3), np.float32)
        st = RtStats()
        _check(lib().rt_renderer_run_host(self.h, pass_begin, count, stride, _ptr(out), C.byref(st)))
        return out, st.as_dict()

    def set_exchange(self, exchange=None, c_fn=None, user=None):
        """Pixel tiles with sort on (rt_renderer_set_exchange).  Either
        exchange(arr): sums the uint8 numpy array over all tile owners in place (host buffer,
        on_device = 0), or c_fn/user: a native rt_exchange_fn (a ctypes function pointer, e.g. from
        a loaded library) called with the device pointer and the pass's HIP stream (on_device = 1),
        which must enqueue its in-place sum on that stream."""
        f = lib().rt_renderer_set_exchange
        if c_fn is not None:
            f.argtypes = [P, P, P, I32]
            self._exchange = (c_fn, user)   # kept alive as long as the renderer
            _check(f(self.h, C.cast(c_fn, P), P(user) if user else None, 1))
            return

        def cb(user, p, n, stream):
            try:
                exchange(np.ctypeslib.as_array(p, shape=(int(n),)))
                return 0
            except Exception:           # reported by the renderer as a failed exchange
                return -1
        self._exchange = EXCHANGE(cb)  # kept alive as long as the renderer
        f.argtypes = [P, EXCHANGE, P, I32]
        _check(f(self.h, self._exchange, None, 0))

    def set_exchange_rccl(self, unique_id, nranks, rank):
        """The exchange over an RCCL communicator the renderer joins (one process per GPU):
        rt_renderer_set_exchange_rccl.  unique_id: the RT_RCCL_ID_BYTES bytes rank 0 got from
        rccl_unique_id(), the same on every rank.  Blocks until every rank has joined."""
        f = lib().rt_renderer_set_exchange_rccl
        f.argtypes = [P, P, I32, I32]
        buf = (C.c_uint8 * RCCL_ID_BYTES).from_buffer_copy(bytes(unique_id))
        _check(f(self.h, buf, int(nranks), int(rank)))

    def set_counters(self, on):
        _check(lib().rt_renderer_set_counters(self.h, int(on)))

    def set_accumulate(self, on):
        """Framebuffer accumulation (rt_renderer_set_accumulate; default on).  Off: runs need d_pass_sums
        and only write them (the multi-GPU drivers add the pass slices themselves)."""
        f = lib().rt_renderer_set_accumulate
        f.argtypes = [P, I32]
        _check(f(self.h, int(on)))

    def launch_profile(self, cap=256):
        """Per trace launch of the last event-timed run's first pass: [(span ms, live rays), ...]
        (rt_renderer_launch_profile)."""
        f = lib().rt_renderer_launch_profile
        f.argtypes = [P, I32, P, P]
        ms = np.zeros(cap, np.float64)
        live = np.zeros(cap, np.uint32)
        n = f(self.h, cap, _ptr(ms), _ptr(live))
        if n < 0:
            _check(n)
        return [(float(ms[b]), int(live[b])) for b in range(n)]

    def set_event_timing(self, on):
        """Per-bounce HIP events for process_ms / sort_ms (default on; off is ~2 % faster)."""
        f = lib().rt_renderer_set_event_timing
        f.argtypes = [P, I32]
        _check(f(self.h, int(on)))

    def framebuffer(self):
        fb = np.zeros(self.scene.pixels * 3, np.float32)
        _check(lib().rt_renderer_read_framebuffer(self.h, _ptr(fb)))
        return fb

    def copy_framebuffer(self, d_out):
        """Device framebuffer -> device pointer d_out (W*H*3 float32 on the renderer's device)."""
        f = lib().rt_renderer_copy_framebuffer
        f.argtypes = [P, P]
        _check(f(self.h, P(d_out)))

    def clear(self):
        _check(lib().rt_renderer_clear(self.h))

    def close(self):
        if getattr(self, "h", None):
            lib().rt_renderer_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def bloom(fb, width, height, threshold, radius=5, device=0):
    out = np.array(fb, dtype=np.float32, copy=True)
    _check(lib().rt_bloom(_ptr(out), width, height, threshold, radius, device))
    return out


def bloom_device(ptr, width, height, threshold, radius=5, device=0):
    _check(lib().rt_bloom_device(P(ptr), width, height, threshold, radius, device))


def tonemap(fb, width, height, exposure, ray_count):
    out = np.zeros(width * height * 3, np.uint8)
    src = np.ascontiguousarray(fb, dtype=np.float32)
    lib().rt_tonemap(_ptr(src), width, height, exposure, ray_count, _ptr(out))
    return out


def write_png(path, rgb, width, height):
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    _check(lib().rt_write_png(path.encode(), _ptr(rgb), width, height))


def cpu_render(scene, threads=0):
    """The reference's `cpu` path (rt_cpu_render). Returns (fb, seconds)."""
    fb = np.zeros(scene.pixels * 3, np.float32)
    secs = C.c_double(0)
    rc = lib().rt_cpu_render(scene.ptr, _ptr(fb), threads, C.byref(secs))
    if rc < 0:
        raise RtError(lib().rt_last_error().decode())
    return fb, secs.value
