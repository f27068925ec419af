"""Model generality on the GPU: the synthetic
tilted-axis robot (tests/golden/tilted_dualarm.urdf: negative and unaligned
joint axes, rotated placements; compiled by ikgrasp/model.py onto canonical
axes) through the generic-path kernels, against oracle/generic_oracle.py's
fixtures (raw axes, np.linalg.pinv loop).

Tolerances: fp64 — identical flags and update counts, q within 1e-9, FK and
frame Jacobians within 1e-12; fp32 — hand error <= 1e-4 against the fp64
targets, update counts within +-2, identical flags."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from helpers import se3_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gc():
    return dict(np.load(os.path.join(GOLDEN, "generic_cases.npz")))


@pytest.fixture(scope="module")
def tilted():
    from ikgrasp.model import DualArmModel
    from ikgrasp.solver import IKSolver
    m = DualArmModel.from_urdf(os.path.join(GOLDEN, "tilted_dualarm.urdf"), os.path.join(GOLDEN, "tilted_cube.urdf"))
    s = IKSolver(m, device=0)
    yield s
    s.close()


def test_solve_fp64_matches_generic_oracle(tilted, gc):
    sol = tilted.solve(gc["targets"], gc["q0"])
    ok = gc["converged"]
    assert np.array_equal(sol.converged, ok) and np.array_equal(sol.iters, gc["iters"])
    assert np.abs(sol.q[ok] - gc["q"][ok]).max() <= 1e-9
    np.testing.assert_allclose(sol.err[ok], gc["err"][ok], atol=1e-10)


def test_solve_fp32_within_ee_tolerance(tilted, gc):
    sol = tilted.solve(gc["targets"], gc["q0"], dtype="f32")
    ok = gc["converged"]
    assert np.array_equal(sol.converged, ok)
    assert (np.abs(sol.iters[ok].astype(int) - gc["iters"][ok]) <= 2).all()
    h32 = tilted.fk(sol.q[ok].astype(np.float64))
    h64 = tilted.fk(gc["q"][ok])
    for h in range(2):  # end-effector SE(3) distance to the fp64 oracle's solution
        e = se3_err(h32[:, h, :9].reshape(-1, 3, 3), h32[:, h, 9:], h64[:, h, :9].reshape(-1, 3, 3), h64[:, h, 9:])
        assert e.max() <= 1e-4


def test_fk_and_frame_jacobian(tilted, gc):
    hands = tilted.fk(gc["fk_q"])
    np.testing.assert_allclose(hands, gc["fk_hands"], atol=1e-12)
    r = tilted.frame_kinematics(gc["fk_q"], None, rf=1, outputs=("placement", "J"))
    np.testing.assert_allclose(r["placement"], gc["fk_hands"], atol=1e-12)
    np.testing.assert_allclose(r["J"], gc["fk_J"], atol=1e-12)


def test_multistart_generic_path(tilted, gc):
    """Best-seed multi-start on the generic path equals the per-seed solves."""
    seeds = np.stack([np.zeros(tilted.nq), gc["q_star"]])
    ms = tilted.solve_multistart(gc["targets"][:8], seeds)
    for t in range(8):
        per = tilted.solve(np.repeat(gc["targets"][t:t + 1], 2, axis=0), seeds)
        b = ms.best_seed[t]
        assert ms.converged[t] == per.converged[b] and np.array_equal(ms.q[t], per.q[b])
