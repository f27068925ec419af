"""Penetration-depth certificate of the collision continuation (DESIGN.md
§3b): epa_depth_lb (ikg_collision.hpp) through the host emulator, against
the support function of A - B sampled by the collision oracle.  The bound
must never exceed the depth (it licenses skipping checks: the answer must not
change), and should be close to it."""
import ctypes as C
import os

import numpy as np

import helpers
import pytest

from ikgrasp import _lib
from oracle import collision_oracle as co


@pytest.fixture(scope="module")
def epa():
    path = helpers.emu_path()
    if not os.path.exists(path):
        pytest.skip("libikgrasp_emu.so not built")
    lib = C.CDLL(path)
    dp = C.POINTER(C.c_double)
    lib.ikg_emu_epa.argtypes = [C.c_int, dp, dp, dp, C.c_int, dp, dp, dp, C.POINTER(C.c_int), dp]

    def run(ga, Ra, ta, gb, Rb, tb):
        arr = lambda x: np.ascontiguousarray(x, dtype=np.float64)
        Ra, ta, da, Rb, tb, db = map(arr, (Ra, ta, ga["dims"], Rb, tb, gb["dims"]))
        p = lambda x: x.ctypes.data_as(dp)
        r, d = C.c_int(), C.c_double()
        lib.ikg_emu_epa(ga["kind"], p(Ra), p(ta), p(da), gb["kind"], p(Rb), p(tb), p(db), C.byref(r), C.byref(d))
        return r.value, d.value

    return run


def _rot(rng):
    Q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
    return Q * np.sign(np.linalg.det(Q))


@pytest.mark.parametrize("ka,kb", [(2, 2), (1, 2), (2, 1), (1, 1)])
def test_epa_bound_is_below_and_near_the_depth(epa, ka, kb):
    rng = np.random.default_rng(10 * ka + kb)
    U = rng.normal(size=(3000, 3))
    U /= np.linalg.norm(U, axis=1, keepdims=True)
    dims = {1: lambda: np.array(rng.uniform(0.02, 0.07, 3)),
            2: lambda: np.array([rng.uniform(0.03, 0.06), rng.uniform(0.015, 0.06), 0.0])}
    n_cert, ratios = 0, []
    for _ in range(40):
        ga = {"kind": ka, "dims": dims[ka]()}
        gb = {"kind": kb, "dims": dims[kb]()}
        Ra, Rb = _rot(rng), _rot(rng)
        ta = np.zeros(3)
        tb = rng.normal(size=3) * 0.05
        r, d = epa(ga, Ra, ta, gb, Rb, tb)
        hit = co.collide(ga, Ra, ta, gb, Rb, tb)
        if not hit:
            assert r == 0
            continue
        assert r >= 1
        if r == 2 and d > 0:
            sa = np.array([co.support(ga, Ra, ta, u) for u in U])
            sb = np.array([co.support(gb, Rb, tb, -u) for u in U])
            depth = np.min(np.sum((sa - sb) * U, axis=1))  # >= the true depth
            assert d <= depth + 1e-12
            n_cert += 1
            ratios.append(d / depth)
    assert n_cert >= 8, n_cert
    print(ka, kb, n_cert, np.round(np.percentile(ratios, [0, 50, 100]), 3))
    assert np.median(ratios) > 0.8
