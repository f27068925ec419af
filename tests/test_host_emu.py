"""Kernel arithmetic on the CPU through the host emulator (ikg_host_emu.hip:
the exact stage functions of ikg_device.hpp composed for both arm lanes).
This is test tooling, not the product path; it lets the CPU suite cover the
specialised (spherical-wrist, compile-time axes) and generic (runtime axes,
Householder QR) solves against the oracle fixtures without a GPU."""
import ctypes as C
import os

import numpy as np

import helpers
import pytest

from ikgrasp import _lib
from ikgrasp.model import load_nextage

EMU = helpers.emu_path()
GENERIC = 99  # ikg_params.variant value the emulator reads as "force the generic path"


@pytest.fixture(scope="module")
def emu():
    if not os.path.exists(EMU):
        pytest.skip("libikgrasp_emu.so not built")
    lib = C.CDLL(EMU)
    vp = C.c_void_p
    lib.ikg_emu_solve.argtypes = [vp, C.c_int, vp, vp, C.c_int64, C.c_int64, vp, vp, vp, vp, vp, vp, C.c_int, vp]
    desc = _lib.model_desc(load_nextage())

    def solve(targets, q0, dtype=0, broadcast=False, **kw):
        npt = np.float64 if dtype == 0 else np.float32
        tg = np.ascontiguousarray(targets, dtype=npt).reshape(-1, 12)
        B = len(tg)
        # per-row q0 (stride 15) runs the kernels' medium-range trig series, a
        # broadcast q0 (stride 0) the short series with the exact fallback
        # (fp64; fp32 takes the medium-range series either way)
        q0 = np.ascontiguousarray(q0 if broadcast else np.broadcast_to(q0, (B, 15)), dtype=npt)
        stride = 0 if broadcast else 15
        p = _lib.default_params(**kw)
        q = np.empty((B, 15), npt)
        conv = np.empty(B, np.uint8)
        it = np.empty(B, np.int32)
        err = np.empty((B, 2), npt)
        assert 0 == lib.ikg_emu_solve(C.byref(desc), dtype, tg.ctypes.data, q0.ctypes.data, stride, B, C.byref(p), q.ctypes.data,
                          conv.ctypes.data, it.ctypes.data, err.ctypes.data, None, 0, None)
        return q, conv.astype(bool), it, err

    return solve


def _kat_targets(kat):
    rows = []
    for k in ("cube_placement", "cube_placement_target"):
        rows.append(np.concatenate([np.array(kat[k]["R"]).reshape(9), kat[k]["t"]]))
    return np.array(rows)


@pytest.mark.parametrize("variant", [0, GENERIC])
def test_emulated_kernel_kats(emu, kat, variant):
    q, conv, it, err = emu(_kat_targets(kat), np.zeros(15), variant=variant)
    assert conv.all() and it.tolist() == [740, 736]
    assert np.abs(q[0] - kat["q0"]).max() <= 1e-12
    assert np.abs(q[1] - kat["qe"]).max() <= 1e-12


@pytest.mark.parametrize("variant", [0, GENERIC])
def test_emulated_kernel_fixtures_fp64(emu, oracle_cases, variant):
    c = oracle_cases
    q, conv, it, err = emu(c["targets"], c["q0"], variant=variant)
    assert np.array_equal(conv, c["converged"]) and np.array_equal(it, c["iters"])
    ok = c["converged"]
    assert np.abs(q[ok] - c["q"][ok]).max() <= 1e-9


def test_emulated_kernel_fp32_kat(emu, kat):
    q, conv, it, err = emu(_kat_targets(kat), np.zeros(15), dtype=1)
    assert conv.all() and (np.abs(it - np.array([740, 736])) <= 2).all()
    assert np.abs(q[0] - kat["q0"]).max() <= 1e-5


def test_emulated_damped_variant_matches_damped_oracle(emu, kat):
    from oracle import ik_oracle as o
    tg = _kat_targets(kat)[:1]
    q, conv, it, err = emu(tg, np.zeros(15), lambda_=1e-4, max_iters=150)
    qo, ok, ito, _ = o.computeqgrasppose(np.zeros(15), np.eye(3), tg[0, 9:], lam=1e-4, max_iters=150)
    assert it[0] == ito and np.abs(q[0] - qo).max() <= 1e-9


@pytest.mark.parametrize("dtype", [0, 1])
def test_medium_trig_series_matches_exact_fallback(emu, dtype):
    """Random seeds take large first steps.  fp64: the medium-range series
    (Trig::step_med, per-problem seeds) and the exact-sincos fallback (broadcast
    q0) must give the same iterates to rounding -- compared over the first 150
    updates, before the non-converging solves' chaotic drift amplifies rounding:
    q within 1e-10.  fp32 runs the medium-range series for both layouts, as the
    kernels do: identical bits."""
    from ikgrasp.workload import random_seeds, uniform_targets
    tg = uniform_targets(6, seed=31)
    for seed in random_seeds(load_nextage(), 3, seed=32):
        a = emu(tg, seed, dtype=dtype, max_iters=150)
        b = emu(tg, seed, dtype=dtype, broadcast=True, max_iters=150)
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
        if dtype == 0:
            assert np.abs(a[0] - b[0]).max() <= 1e-10
        else:
            assert np.array_equal(a[0], b[0])


def _emu_math(fn, x, y=None):
    lib = C.CDLL(EMU)
    lib.ikg_emu_math.argtypes = [C.c_int, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(x if y is None else y, dtype=np.float64)
    out = np.empty(2 * len(x), dtype=np.float64)
    assert lib.ikg_emu_math(fn, len(x), x.ctypes.data, y.ctypes.data, out.ctypes.data) == 0
    return out


def test_loop_math_accuracy():
    """The loop's own math (ikg_device.hpp): Cody-Waite sincos within 2 ulp
    (fp64) / 2 ulp of float (fp32) over the joint range and beyond, and the
    packed pair's atan2_upper within 1.5 float ulps of pi (3.6e-7) over the
    upper half plane (host arithmetic: exact division instead of the device's
    reciprocal refinement)."""
    if not os.path.exists(EMU):
        pytest.skip("libikgrasp_emu.so not built")
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(-8, 8, 20000), np.linspace(-np.pi, np.pi, 4001), [0.0, 1e-300, -1e-300]])
    o = _emu_math(0, x).reshape(-1, 2)
    assert np.abs(o[:, 0] - np.sin(x)).max() <= 2 * np.spacing(1.0)
    assert np.abs(o[:, 1] - np.cos(x)).max() <= 2 * np.spacing(1.0)
    xf = x.astype(np.float32).astype(np.float64)
    for fn in (1, 2):
        o = _emu_math(fn, xf).reshape(-1, 2)
        assert np.abs(o[:, 0] - np.sin(xf)).max() <= 2 * float(np.spacing(np.float32(1.0)))
        assert np.abs(o[:, 1] - np.cos(xf)).max() <= 2 * float(np.spacing(np.float32(1.0)))
    th = np.concatenate([rng.uniform(0, np.pi, 20000), [0.0, np.pi / 4, np.pi / 2, np.pi, 1e-6, np.pi - 1e-6]])
    r = rng.uniform(0.5, 2.0, len(th))
    yy = (r * np.sin(th)).astype(np.float32).astype(np.float64)
    xx = (r * np.cos(th)).astype(np.float32).astype(np.float64)
    for fn in (3, 4):
        a = _emu_math(fn, xx, yy)[:len(xx)]
        assert np.abs(a - np.arctan2(yy, xx)).max() <= 1.5 * float(np.spacing(np.float32(np.pi)))


def test_emulated_kernel_sensitive_cases(emu):
    """Rounding-sensitive random-seed trajectories (tests/golden/
    sensitive_cases.npz): flags and update counts equal the 32-digit loop's, and
    q is within 1e-9 of it -- or, where float64 itself cannot get there, no
    farther than the reference's own answer is plus the reference's rounding
    envelope."""
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "sensitive_cases.npz"))
    q, conv, it, err = emu(d["targets"], d["q0"])
    assert np.array_equal(conv, d["converged_exact"]) and np.array_equal(it, d["iters_exact"])
    gpu = np.abs(q - d["q_exact"]).max(axis=1)
    ref = np.abs(d["q"] - d["q_exact"]).max(axis=1)
    print("kernel (emulated) vs exact", gpu, "\nnumpy reference vs exact", ref)
    assert (gpu <= np.maximum(1e-9, ref + d["envelope"])).all()
