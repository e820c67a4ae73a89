"""ctypes loader of tests/native/build/libxchg.so — TEST / PROBE INFRASTRUCTURE (tests/native/xchg.hip):
device-side pixel-tile bucket-byte exchanges for a host with one GPU (the multi-GPU library path
uses RCCL's ncclAllReduce instead)."""
import ctypes as C
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(REPO, "tests", "native")
LIB_PATH = os.path.join(NATIVE, "build", "libxchg.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-s", "-C", NATIVE], check=True)
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.xchg_group_create.restype = P
        L.xchg_group_create.argtypes = [C.c_int]
        L.xchg_group_member.restype = P
        L.xchg_group_member.argtypes = [P, C.c_int]
        L.xchg_group_destroy.argtypes = [P]
        L.xchg_emulate_create.restype = P
        L.xchg_emulate_destroy.argtypes = [P]
        _lib = L
    return _lib


class Group:
    """Tile owners on one device summing their bytes device-side (xchg_group_fn)."""

    def __init__(self, owners):
        self.h = lib().xchg_group_create(owners)
        if not self.h:
            raise RuntimeError("xchg_group_create failed")

    def attach(self, renderer, rank):
        renderer.set_exchange(c_fn=lib().xchg_group_fn, user=lib().xchg_group_member(self.h, rank))

    def close(self):
        if self.h:
            lib().xchg_group_destroy(self.h)
            self.h = None


class EmulatedPeers:
    """One owner alone; the absent owners' global slots emulated (xchg_emulate_peers)."""

    def __init__(self):
        self.h = lib().xchg_emulate_create()
        if not self.h:
            raise RuntimeError("xchg_emulate_create failed")

    def attach(self, renderer):
        renderer.set_exchange(c_fn=lib().xchg_emulate_peers, user=self.h)

    def close(self):
        if self.h:
            lib().xchg_emulate_destroy(self.h)
            self.h = None
