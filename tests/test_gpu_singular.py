"""pinv semantics at arm-block singularities on the MI355X (the CPU side and
the fixtures are described in tests/test_singular.py).

fp64 (pair kernel): flags and update counts identical to the exact-pinv loop
on all 48 cases, q within max(1e-9, 2e-19 cond(J)); identical to the numpy
oracle where cond(J) < 1e6, q within 1e-9.  fp32 (pair and packed layouts):
where cond(J) < 1e6, flags identical, updates within +-2 and end-effector
error <= 1e-4 per hand for converged solves.  The guard's LQ branch is also
run on every update (IKG_SING_BETA=0) against the ordinary fixtures, in the
batch, multi-start and collision paths."""
import os

import numpy as np
import pytest

import helpers
from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sing():
    return dict(np.load(os.path.join(GOLDEN, "singular_cases.npz")))


def _ee_ok(solver, q_gpu, q_ref, mask, tol=1e-4):
    hg = solver.fk(q_gpu[mask].astype(np.float64))
    ho = solver.fk(q_ref[mask])
    for h in range(2):
        e = helpers.se3_err(ho[:, h, :9].reshape(-1, 3, 3), ho[:, h, 9:], hg[:, h, :9].reshape(-1, 3, 3), hg[:, h, 9:])
        assert e.max() <= tol


def test_singular_seeds_fp64(solver, sing):
    c = sing
    sol = solver.solve(c["targets"], c["q0"], dtype="f64")
    assert np.array_equal(sol.converged, c["converged_exact"]) and np.array_equal(sol.iters, c["iters_exact"])
    assert (np.abs(sol.q - c["q_exact"]).max(axis=1) <= np.maximum(1e-9, 2e-19 * c["cond0"])).all()
    well = c["cond0"] < 1e6
    assert np.array_equal(sol.converged[well], c["converged"][well])
    assert np.array_equal(sol.iters[well], c["iters"][well])
    assert np.abs(sol.q[well] - c["q"][well]).max() <= 1e-9


@pytest.mark.parametrize("variant", ["pair", "packed"])
def test_singular_seeds_fp32(solver, sing, variant):
    from ikgrasp import _lib
    c = sing
    v = _lib.IKG_VARIANT_PAIR if variant == "pair" else _lib.IKG_VARIANT_PACKED
    sol = solver.solve(c["targets"], c["q0"], dtype="f32", variant=v)
    well = c["cond0"] < 1e6
    assert np.array_equal(sol.converged[well], c["converged"][well])
    both = well & sol.converged
    assert np.abs(sol.iters[both].astype(int) - c["iters"][both]).max() <= 2
    _ee_ok(solver, sol.q, c["q"], both)


@pytest.fixture(scope="module")
def lq_solver():
    """A solver whose tables were built with IKG_SING_BETA=0: every update
    takes the guard's LQ branch."""
    from ikgrasp.collision import load_nextage_scene
    from ikgrasp.solver import IKSolver
    old = os.environ.get("IKG_SING_BETA")
    os.environ["IKG_SING_BETA"] = "0"
    try:
        s = IKSolver(device=0, scene=load_nextage_scene())
        s.solve(np.zeros((1, 12)) + np.concatenate([np.eye(3).ravel(), [0.4, 0.1, 0.93]]), np.zeros(15))
        s.solve(np.zeros((1, 12)) + np.concatenate([np.eye(3).ravel(), [0.4, 0.1, 0.93]]), np.zeros(15), dtype="f32")
    finally:
        if old is None:
            del os.environ["IKG_SING_BETA"]
        else:
            os.environ["IKG_SING_BETA"] = old
    yield s
    s.close()


def test_lq_branch_everywhere_fp64(lq_solver, oracle_cases):
    c = oracle_cases
    sol = lq_solver.solve(c["targets"], c["q0"], dtype="f64")
    assert np.array_equal(sol.converged, c["converged"]) and np.array_equal(sol.iters, c["iters"])
    conv = c["converged"]
    assert np.abs(sol.q[conv] - c["q"][conv]).max() <= 1e-9


@pytest.mark.parametrize("variant", ["pair", "packed", "quad"])
def test_lq_branch_everywhere_fp32(lq_solver, oracle_cases, variant):
    from ikgrasp import _lib
    c = oracle_cases
    v = {"pair": _lib.IKG_VARIANT_PAIR, "packed": _lib.IKG_VARIANT_PACKED, "quad": _lib.IKG_VARIANT_QUAD}[variant]
    sol = lq_solver.solve(c["targets"], c["q0"], dtype="f32", variant=v)
    assert np.array_equal(sol.converged, c["converged"])
    both = c["converged"] & sol.converged
    assert np.abs(sol.iters[both].astype(int) - c["iters"][both]).max() <= 2
    _ee_ok(lq_solver, sol.q, c["q"], both)


def test_lq_branch_everywhere_quad_fp64(lq_solver, oracle_cases):
    from ikgrasp import _lib
    c = oracle_cases
    sol = lq_solver.solve(c["targets"], c["q0"], dtype="f64", variant=_lib.IKG_VARIANT_QUAD)
    assert np.array_equal(sol.converged, c["converged"]) and np.array_equal(sol.iters, c["iters"])
    assert np.abs(sol.q[c["converged"]] - c["q"][c["converged"]]).max() <= 1e-9


def test_lq_branch_everywhere_with_collision(lq_solver):
    """The collision continuation's steps (records in the batch kernel, the
    trajectory kernel for per-problem seeds, the interleaved continuation)
    through the LQ branch: the collision fixtures' flags and counts."""
    c = dict(np.load(os.path.join(GOLDEN, "collision_solve_cases.npz")))
    sol = lq_solver.solve(c["targets"], c["q0"], check_collision=True)
    assert np.array_equal(sol.converged, c["success"]) and np.array_equal(sol.iters, c["iters"])
    s = c["success"]
    assert np.abs(sol.q[s] - c["q"][s]).max() <= 1e-9
    os.environ["IKG_CONT_TRAJ"] = "0"
    try:
        sol2 = lq_solver.solve(c["targets"], c["q0"], check_collision=True)
    finally:
        del os.environ["IKG_CONT_TRAJ"]
    assert np.array_equal(sol2.converged, c["success"]) and np.array_equal(sol2.iters, c["iters"])


def test_multistart_with_singular_seeds(solver, sing):
    """Seeds at the singularities in a multi-start solve: the winner equals
    the argmin over the expanded batch solve, bit for bit."""
    c = sing
    seeds = np.unique(c["q0"], axis=0)
    tg = c["targets"][:16]
    ms = solver.solve_multistart(tg, seeds)
    S = len(seeds)
    ex = solver.solve(np.repeat(tg, S, axis=0), np.tile(seeds, (len(tg), 1)))
    for t in range(len(tg)):
        rows = slice(t * S, (t + 1) * S)
        conv = ex.converged[rows]
        key = np.where(conv, np.max(ex.err[rows], axis=1), np.inf)
        if conv.any():
            b = int(np.argmin(key))
            assert ms.best_seed[t] == b
            assert np.array_equal(ms.q[t], ex.q[rows][b])
        else:
            assert not ms.converged[t]
