"""pinv semantics at arm-block singularities (inverse_geometry.py:83,
np.linalg.pinv(J) @ e), CPU side: the fixtures themselves and the kernel's
arithmetic through the host emulator (the exact device stage functions).

`tests/golden/singular_cases.npz` (make_golden.py singular): seeds at and
1e-9 / 1e-6 / 1e-3 rad from the wrist (arm joint 4 at -pi/2), straight-elbow
and shoulder (wrist centre on arm joint 0's axis) singularities of each arm,
two targets each, solved by the numpy oracle and by the same loop with a
40-digit pinv step (`pinv_exact`).

Gates (fp64): flags and update counts identical to the exact-pinv loop on
every case and q within max(1e-9, 2e-19 cond(J)) (the kernel's own rounding
at cond(J) = 1.75e10 is 1.3e-9); identical to the numpy oracle wherever
cond(J) < 1e6, q within 1e-9.  Where J itself is ill-conditioned (the
straight elbow: the chest cannot restore the lost direction), numpy's own
result is off the exact one by up to 1.3 rad (LAPACK rounding amplified by
cond(J); on the first step it puts 79 rad into the exactly-zero head
columns), so no implementation can match it there bit for bit.
"""
import ctypes as C
import os

import numpy as np
import pytest

import helpers
from conftest import GOLDEN
from ikgrasp import _lib
from ikgrasp.model import load_nextage

EMU = helpers.emu_path()


@pytest.fixture(scope="module")
def sing():
    return dict(np.load(os.path.join(GOLDEN, "singular_cases.npz")))


@pytest.fixture(scope="module")
def emu():
    if not os.path.exists(EMU):
        pytest.skip("libikgrasp_emu.so not built")
    lib = C.CDLL(EMU)
    vp = C.c_void_p
    lib.ikg_emu_solve.argtypes = [vp, C.c_int, vp, vp, C.c_int64, C.c_int64, vp, vp, vp, vp, vp, vp, C.c_int, vp]
    lib.ikg_emu_lq_count.restype = C.c_longlong
    lib.ikg_emu_svd_count.restype = C.c_longlong
    desc = _lib.model_desc(load_nextage())

    def solve(targets, q0, dtype=0):
        npt = np.float64 if dtype == 0 else np.float32
        tg = np.ascontiguousarray(targets, dtype=npt)
        B = len(tg)
        q0 = np.ascontiguousarray(q0, dtype=npt)
        p = _lib.default_params()
        q = np.empty((B, 15), npt)
        conv = np.empty(B, np.uint8)
        it = np.empty(B, np.int32)
        err = np.empty((B, 2), npt)
        assert 0 == lib.ikg_emu_solve(C.byref(desc), dtype, tg.ctypes.data, q0.ctypes.data, 15, B, C.byref(p), q.ctypes.data,
                          conv.ctypes.data, it.ctypes.data, err.ctypes.data, None, 0, None)
        return q, conv.astype(bool), it

    solve.lib = lib
    return solve


def tol_exact(cond0):
    return np.maximum(1e-9, 2e-19 * cond0)


def test_fixture_seeds_sit_at_the_singularities(sing):
    from oracle import ik_oracle as o
    at = sing["delta"] == 0.0
    for q0, arm in zip(sing["q0"][at], sing["arm"][at]):
        J = o.frame_jacobian_local(q0, o.FRAME_LEFT if arm == 0 else o.FRAME_RIGHT)
        cols = slice(3, 9) if arm == 0 else slice(9, 15)
        s = np.linalg.svd(J[:, cols], compute_uv=False)
        assert s[-1] < 1e-9 * s[0]  # the 6 x 6 arm block is singular


def test_numpy_oracle_equals_exact_pinv_where_j_is_well_conditioned(sing):
    c = sing
    well = c["cond0"] < 1e6
    assert well.sum() >= 32 and (~well).sum() >= 8
    assert np.array_equal(c["converged"][well], c["converged_exact"][well])
    assert np.array_equal(c["iters"][well], c["iters_exact"][well])
    assert np.abs(c["q"][well] - c["q_exact"][well]).max() <= 1e-10


def test_emulated_kernel_matches_pinv_at_singularities(emu, sing):
    c = sing
    emu.lib.ikg_emu_lq_count(1)
    emu.lib.ikg_emu_svd_count(1)
    q, conv, it = emu(c["targets"], c["q0"])
    assert emu.lib.ikg_emu_lq_count(1) >= 16  # the guard took the LQ form
    assert emu.lib.ikg_emu_svd_count(1) >= 2  # and the Jacobi form at the exact straight elbows
    assert np.array_equal(conv, c["converged_exact"]) and np.array_equal(it, c["iters_exact"])
    assert (np.abs(q - c["q_exact"]).max(axis=1) <= tol_exact(c["cond0"])).all()
    well = c["cond0"] < 1e6
    assert np.array_equal(conv[well], c["converged"][well]) and np.array_equal(it[well], c["iters"][well])
    assert np.abs(q[well] - c["q"][well]).max() <= 1e-9


def test_emulated_kernel_fp32_at_singularities(emu, sing):
    c = sing
    well = c["cond0"] < 1e6
    q, conv, it = emu(c["targets"], c["q0"], dtype=1)
    assert np.array_equal(conv[well], c["converged"][well])
    both = well & conv
    assert np.abs(it[both] - c["iters"][both]).max() <= 2
    m = load_nextage()
    for i in np.nonzero(both)[0]:
        hg, ho = helpers.hands_from_tables(m, q[i].astype(np.float64)), helpers.hands_from_tables(m, c["q"][i])
        for h in range(2):
            e = helpers.se3_err(ho[None, h, :9].reshape(1, 3, 3), ho[None, h, 9:],
                                hg[None, h, :9].reshape(1, 3, 3), hg[None, h, 9:])
            assert e[0] <= 1e-4


def test_lq_form_everywhere_reproduces_the_fixtures(emu, oracle_cases, monkeypatch):
    """IKG_SING_BETA=0 sends every update through the LQ form (the guard's
    branch): the 96 oracle fixtures come out as with the closed form."""
    monkeypatch.setenv("IKG_SING_BETA", "0")
    c = oracle_cases
    emu.lib.ikg_emu_lq_count(1)
    q, conv, it = emu(c["targets"], c["q0"])
    assert emu.lib.ikg_emu_lq_count(1) == int(c["iters"].sum())
    assert np.array_equal(conv, c["converged"]) and np.array_equal(it, c["iters"])
    assert np.abs(q[conv] - c["q"][conv]).max() <= 1e-9
