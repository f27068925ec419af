"""The C restatement (oracle/ikg_oracle.c) — bench.py's CPU baseline legs —
pinned against the golden fixtures, like the Python oracles it restates:

* the plain loop (inverse_geometry.py:41-100 without :70's collision term)
  against tests/golden/oracle_cases.npz (numpy oracle, itself pinned by the
  reference's KATs, make_golden.py);
* tools.collision (tools.py:25-35) against tests/golden/collision_cases.npz
  (oracle/collision_oracle.py's verdicts, 1475 configurations);
* the loop WITH the collision term (:70, :97-98) against
  tests/golden/collision_solve_cases.npz.

CPU only: the C oracle is test / baseline infrastructure, never the product.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import c_oracle, collision_oracle  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")

pytestmark = pytest.mark.skipif(not os.path.exists(c_oracle.LIB), reason="oracle/_build not built (make -C oracle)")


@pytest.fixture(scope="module")
def scene():
    return collision_oracle.load_scene(os.path.join(GOLD, "collision_scene.json"))


def test_plain_loop_matches_golden():
    d = np.load(os.path.join(GOLD, "oracle_cases.npz"))
    q, conv, iters, err = c_oracle.solve(d["targets"], d["q0"], threads=2)
    assert (conv == d["converged"]).all()
    assert (iters == d["iters"]).all()
    np.testing.assert_allclose(q, d["q"], atol=1e-9, rtol=0)


def test_collision_term_matches_golden(scene):
    d = np.load(os.path.join(GOLD, "collision_cases.npz"))
    c = c_oracle.collision(scene, d["q"], d["targets"])
    mism = int((c != d["collision"]).sum())
    print(f"C collision vs collision_cases.npz: {mism} mismatches of {len(c)} ({int(c.sum())} colliding)")
    assert mism == 0


def test_collision_solve_matches_golden(scene):
    d = np.load(os.path.join(GOLD, "collision_solve_cases.npz"))
    q, ok, iters, err = c_oracle.solve_collision(scene, d["targets"], d["q0"], threads=2)
    assert (ok == d["success"]).all()
    assert (iters == d["iters"]).all()
    np.testing.assert_allclose(q, d["q"], atol=1e-9, rtol=0)
    np.testing.assert_allclose(err, d["err"], atol=1e-9, rtol=0)


def test_collision_solve_without_pairs_is_plain_loop(scene):
    """An empty pair list makes :70's collision term always false."""
    d = np.load(os.path.join(GOLD, "oracle_cases.npz"))
    empty = dict(scene, pairs=[])
    q1, c1, i1, _ = c_oracle.solve_collision(empty, d["targets"][:24], d["q0"][:24])
    q2, c2, i2, _ = c_oracle.solve(d["targets"][:24], d["q0"][:24])
    assert (c1 == c2).all() and (i1 == i2).all()
    assert np.array_equal(q1, q2)


# ---------------------------------------------------------------- evaluation modes
def _kat_rows(kat):
    return np.array([np.concatenate([np.array(kat[k]["R"]).reshape(9), kat[k]["t"]])
                     for k in ("cube_placement", "cube_placement_target")])


@pytest.mark.parametrize("flags", [0, c_oracle.ACC_LOG6, c_oracle.QR_STEP, c_oracle.ACC_LOG6 | c_oracle.QR_STEP,
                                   c_oracle.QR_STEP | c_oracle.JITTER])
def test_oracle_modes_reproduce_kats(kat, flags):
    """Every evaluation mode is the same loop: KAT-1/2 (trajectory.json) in
    740/736 updates.  These two trajectories are well conditioned, so even the
    1-ulp FK jitter leaves q within a few ulp."""
    q, conv, iters, _ = c_oracle.solve_ex(_kat_rows(kat), np.zeros(15), flags, seed=3)
    assert conv.all() and iters.tolist() == [740, 736]
    assert np.abs(q[0] - kat["q0"]).max() <= 1e-14 and np.abs(q[1] - kat["qe"]).max() <= 1e-14


def test_sensitive_cases_rounding_envelope():
    """tests/golden/sensitive_cases.npz: on rounding-sensitive random-seed
    trajectories the reference's own float64 answer (numpy: pinv step,
    Pinocchio's acos log6) is only defined up to its rounding envelope, and the
    loop evaluated without log6's cancellation (C oracle ACC_LOG6 | QR_STEP)
    lands at least as close to the 32-digit loop as the reference does."""
    d = np.load(os.path.join(GOLD, "sensitive_cases.npz"))
    assert np.array_equal(d["converged"], d["converged_exact"]) and np.array_equal(d["iters"], d["iters_exact"])
    # the QR step with the reference's log6 reproduces numpy's answer within the envelope
    q, c, it, _ = c_oracle.solve_ex(d["targets"], d["q0"], c_oracle.QR_STEP)
    assert np.array_equal(c, d["converged"]) and np.array_equal(it, d["iters"])
    assert (np.abs(q - d["q"]).max(axis=1) <= np.maximum(1e-9, 2 * d["envelope"])).all()
    qa, ca, ia, _ = c_oracle.solve_ex(d["targets"], d["q0"], c_oracle.ACC_LOG6 | c_oracle.QR_STEP)
    assert np.array_equal(ca, d["converged_exact"]) and np.array_equal(ia, d["iters_exact"])
    ref = np.abs(d["q"] - d["q_exact"]).max(axis=1)
    acc = np.abs(qa - d["q_exact"]).max(axis=1)
    print("numpy vs exact", ref, "\nC acc vs exact", acc, "\nenvelope", d["envelope"])
    assert (acc <= np.maximum(1e-9, ref + d["envelope"])).all()
    assert ref.max() > 1e-8  # the fixture does hold cases where the reference's own answer is off by > 1e-8
