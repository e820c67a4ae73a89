"""The oracle's analysis-only models (tools/chain_models.py, tools/route_model.py): invariants on a small scene.
They are not on the parity path; these checks keep the numbers DESIGN.md §5 quotes from silently breaking."""
import ctypes as C
import os

import numpy as np

import oracle_lib as O


def _scene():
    return O.OracleScene(os.path.join(O.ASSETS, "cornell.scene"), image=(64, 64, 20, 4))


def test_route_model_invariants():
    sc, L = _scene(), O.lib()
    L.orc_bounce_working_set.argtypes = [C.c_void_p] + [C.c_int] * 6 + [C.c_void_p, C.c_int]
    out = np.zeros(21)
    assert L.orc_bounce_working_set(sc.h, 1, 0, 1, 512, 2, 4, out.ctypes.data_as(C.c_void_p), 2) == 0
    pol = out[:18].reshape(3, 6)
    assert pol[0, 5] > 0 and pol[0, 5] == pol[1, 5] == pol[2, 5]    # the same rays fetch the same bytes
    live = out[19]
    assert live > 0 and 0 <= out[20] <= live
    assert pol[0, 3] <= (np.ceil(live / 8) + 1) / live                # eighths: balanced to a ray,
    assert pol[1, 3] <= (np.ceil(live / 8) + 65) / live               # or to a ray per bucket
    for p in pol:
        assert 0 < p[0] <= p[1] and 0 <= p[4] <= p[5] and 0 < p[3] <= 1
    bad = np.zeros(21)
    assert L.orc_bounce_working_set(sc.h, 1, 0, 4, 512, 2, 4, bad.ctypes.data_as(C.c_void_p), 2) != 0   # no bounce 4
    assert L.orc_bounce_working_set(sc.h, 1, 0, 1, 0, 2, 4, bad.ctypes.data_as(C.c_void_p), 2) != 0     # window 0


def test_chain_profile_models_order():
    """Two-level records never need more fetches than one-level ones (tools/chain_models.py's cur >= tl1 >= tl2)."""
    sc, L = _scene(), O.lib()
    L.orc_pass_chain_profile.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int]
    a = np.zeros((4, 8), np.uint64)
    assert L.orc_pass_chain_profile(sc.h, 1, 0, a.ctypes.data_as(C.c_void_p), 2) == 0
    assert a[0, 4] > 0
    assert np.all(a[:, 4] >= a[:, 5]) and np.all(a[:, 5] >= a[:, 6]) and np.all(a[:, 7] >= a[:, 5])
    assert np.all(a[:, 0] >= a[:, 1])


def test_wave_model_invariants():
    """Re-ordering rays inside tiles changes which rays share a wave, never the work (tools/wave_model.py)."""
    sc, L = _scene(), O.lib()
    L.orc_bounce_wave_model.argtypes = [C.c_void_p] + [C.c_int] * 7 + [C.c_void_p, C.c_int]
    out = np.zeros(12)
    assert L.orc_bounce_wave_model(sc.h, 1, 0, 1, 256, 4, 2, 24, out.ctypes.data_as(C.c_void_p), 2) == 0
    a, b = out[:6], out[6:]
    assert a[3] > 0 and a[3] == b[3] and a[5] == b[5]               # same lane-steps, same longest ray
    for o in (a, b):
        assert o[0] > 0 and o[1] <= o[0] and o[2] <= o[0] and o[1] + o[2] >= o[0]
        assert o[3] <= 64 * (o[1] + o[2])
    assert L.orc_bounce_wave_model(sc.h, 1, 0, 1, 256, 4, 2, 0, out.ctypes.data_as(C.c_void_p), 2) != 0   # refill 0
