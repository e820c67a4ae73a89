"""ctypes bindings for the parity oracle (oracle/build/liboracle.so) — TEST INFRASTRUCTURE ONLY."""
import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
# ORACLE_LIB: another build of the oracle (tools/fastmath_floor.py: build/liboracle_fastmath.so)
LIB_PATH = os.environ.get("ORACLE_LIB") or os.path.join(ORACLE_DIR, "build", "liboracle.so")
ASSETS = os.path.join(REPO, "assets")


class OrcInfo(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("width", "height", "ray_count", "bounces")] + \
               [("exposure", C.c_float)] + \
               [(n, C.c_int32) for n in ("sphere_count", "triangle_count", "material_count",
                                         "bvh_node_count", "env_width", "env_height")]


class OrcStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "generated_rays", "live_segments", "dead_slots", "nodes_popped", "internal_visits",
        "triangle_tests", "sphere_tests", "hits_triangle", "hits_sphere", "misses",
        "sorted_items")] + [("max_stack", C.c_uint32), ("passes", C.c_uint32),
                                     ("max_ray_nodes", C.c_uint32), ("reserved", C.c_uint32)]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


_lib = None



EXCHANGE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint8), C.c_int64)

def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.orc_load_scene.restype = P
        L.orc_load_scene.argtypes = [C.c_char_p, C.c_int, C.c_char_p, P, P]
        L.orc_free_scene.argtypes = [P]
        L.orc_last_error.restype = C.c_char_p
        L.orc_get_info.argtypes = [P, P]
        L.orc_get_arrays.argtypes = [P] * 8
        L.orc_render_gpu_semantics.argtypes = [P, C.c_int, C.c_int, C.c_int, P, P, P, C.c_int]
        L.orc_render_pass_sums.argtypes = [P, C.c_int, C.c_int, C.c_int, P, C.c_int]
        L.orc_render_tiled.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, EXCHANGE, P, P, P,
                                       C.c_int]
        L.orc_render_cpu_path.argtypes = [P, P, C.c_int, C.c_int, P]
        L.orc_closest_hit.argtypes = [P, P, C.c_int, P, P, P]
        L.orc_pass_bounce_profile.argtypes = [P, C.c_int, C.c_int, P, P, C.c_int]
        L.orc_bloom.argtypes = [P, C.c_int, C.c_int, C.c_float, C.c_int]
        L.orc_tonemap.argtypes = [P, C.c_int, C.c_int, C.c_float, C.c_int, P]
        L.orc_pcg_stream.argtypes = [C.c_uint32, C.c_int, P]
        L.orc_random_draws.argtypes = [C.c_uint32, C.c_int, P, P, P]
        L.orc_random_on_sphere.argtypes = [C.c_uint32, C.c_int, P]
        L.orc_sincos.argtypes = [P, C.c_int, P, P]
        L.orc_atan01.argtypes = [C.c_float]
        L.orc_atan01.restype = C.c_float
        for n in ("orc_generate_seed", "orc_process_seed", "orc_cpu_seed"):
            getattr(L, n).argtypes = [C.c_int32, C.c_int32]
            getattr(L, n).restype = C.c_uint32
        L.orc_interleave_5.argtypes = [C.c_uint16]
        L.orc_interleave_5.restype = C.c_uint16
        L.orc_morton.argtypes = [C.c_float] * 3
        L.orc_morton.restype = C.c_uint32
        L.orc_key_bucket.argtypes = [C.c_uint32]
        L.orc_ray_aabb.argtypes = [P, P, P, P, C.c_float, P]
        L.orc_ray_triangle.argtypes = [P, P, P, C.c_float, P]
        L.orc_ray_sphere.argtypes = [P, P, P, C.c_float, P]
        L.orc_env_project.argtypes = [P, P]
        L.orc_env_texel.argtypes = [P, C.c_int, C.c_int]
        _lib = L
    return _lib


def ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class OracleScene:
    """A scene loaded by the oracle's own restated loader + BVH builder."""

    def __init__(self, path, use_bvh=True, asset_root=ASSETS, image=None, exposure=None):
        L = lib()
        img = np.asarray(image, dtype=np.int32) if image is not None else None
        exp = np.asarray([exposure], dtype=np.float32) if exposure is not None else None
        self.h = L.orc_load_scene(path.encode(), int(use_bvh),
                                  asset_root.encode() if asset_root else None, ptr(img), ptr(exp))
        if not self.h:
            raise RuntimeError(L.orc_last_error().decode())
        self.info = OrcInfo()
        L.orc_get_info(self.h, C.byref(self.info))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_free_scene(self.h)
            self.h = None

    @property
    def pixels(self):
        return self.info.width * self.info.height

    @property
    def passes(self):
        return (self.info.ray_count + 19) // 20

    def arrays(self):
        i = self.info
        sph = np.zeros((i.sphere_count, 4), np.float32)
        tri = np.zeros((i.triangle_count, 12), np.float32)
        mi = np.zeros(i.sphere_count + i.triangle_count, np.uint16)
        mat = np.zeros((i.material_count, 12), np.float32)
        bvh = np.zeros((i.bvh_node_count, 8), np.float32)
        env = np.zeros((i.env_width * i.env_height, 3), np.float32)
        cam = np.zeros(30, np.float32)
        lib().orc_get_arrays(self.h, ptr(sph), ptr(tri), ptr(mi), ptr(mat), ptr(bvh), ptr(env), ptr(cam))
        return dict(spheres=sph, triangles=tri, material_indices=mi, materials=mat,
                    bvh=bvh, env=env, camera=cam)

    def render(self, sort=True, pass_begin=0, pass_count=-1, threads=0, hist=False):
        fb = np.zeros(self.pixels * 3, np.float32)
        st = OrcStats()
        n = self.passes - pass_begin if pass_count < 0 else pass_count
        h = np.zeros((n, self.info.bounces, 65), np.uint64) if hist else None
        rc = lib().orc_render_gpu_semantics(self.h, int(sort), pass_begin, pass_count, ptr(fb),
                                            C.byref(st), ptr(h), threads)
        if rc != 0:
            raise RuntimeError(lib().orc_last_error().decode())
        return (fb, st.as_dict(), h) if hist else (fb, st.as_dict())

    def bounce_profile(self, sort=True, pass_index=0, threads=0):
        """Per bounce of one pass: (longest ray's trace steps = internal visits + triangle tests,
        live rays) -- orc_pass_bounce_profile."""
        steps = np.zeros(self.info.bounces, np.uint32)
        live = np.zeros(self.info.bounces, np.uint64)
        rc = lib().orc_pass_bounce_profile(self.h, int(sort), pass_index, ptr(steps), ptr(live), threads)
        if rc:
            raise RuntimeError(lib().orc_last_error().decode())
        return steps, live

    def pass_sums(self, sort=True, pass_begin=0, pass_count=1, threads=0):
        out = np.zeros((pass_count, self.pixels * 3), np.float32)
        rc = lib().orc_render_pass_sums(self.h, int(sort), pass_begin, pass_count, ptr(out), threads)
        if rc != 0:
            raise RuntimeError(lib().orc_last_error().decode())
        return out

    def render_tiled(self, exchange, tile_count, tile_index, tile_rows=8, sort=True, pass_begin=0, pass_count=-1,
                     threads=0):
        """orc_render_tiled: this owner's row stripes only, with the per-bounce bucket exchange
        (SURVEY §8e sort on).  exchange(arr) must sum the uint8 array over all owners in place.
        Returns (fb with this owner's pixels, others 0; stats)."""
        fb = np.zeros(self.pixels * 3, np.float32)
        st = OrcStats()

        def cb(user, p, n):
            try:
                exchange(np.ctypeslib.as_array(p, shape=(n,)))
                return 0
            except Exception:       # reported as a failed exchange by the oracle
                return -1
        fn = EXCHANGE(cb)
        rc = lib().orc_render_tiled(self.h, int(sort), tile_count, tile_index, tile_rows, pass_begin, pass_count, fn,
                                    None, ptr(fb), C.byref(st), threads)
        if rc != 0:
            raise RuntimeError(lib().orc_last_error().decode())
        return fb, st.as_dict()

    def closest_hit(self, rays):
        """Closest hit of rays (n, 6) {o.xyz, d.xyz}: (t, index, stats)."""
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        t = np.zeros(rays.shape[0], np.float32)
        idx = np.zeros(rays.shape[0], np.int32)
        st = OrcStats()
        lib().orc_closest_hit(self.h, ptr(rays), rays.shape[0], ptr(t), ptr(idx), C.byref(st))
        return t, idx, st.as_dict()

    def render_cpu_path(self, pass_limit=-1, threads=0):
        fb = np.zeros(self.pixels * 3, np.float32)
        secs = C.c_double(0)
        lib().orc_render_cpu_path(self.h, ptr(fb), pass_limit, threads, C.byref(secs))
        return fb, secs.value


def bloom(fb, w, h, threshold, radius=5):
    out = np.array(fb, dtype=np.float32, copy=True)
    lib().orc_bloom(ptr(out), w, h, threshold, radius)
    return out


def tonemap(fb, w, h, exposure, ray_count):
    out = np.zeros(w * h * 3, np.uint8)
    src = np.ascontiguousarray(fb, dtype=np.float32)
    lib().orc_tonemap(ptr(src), w, h, exposure, ray_count, ptr(out))
    return out
