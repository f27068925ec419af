"""The oracle is pinned to the reference's own known answers before it is
trusted as the checker."""
import numpy as np
import pytest

from oracle import ik_oracle as o


def _placement(d):
    return np.array(d["R"], dtype=np.float64), np.array(d["t"], dtype=np.float64)


@pytest.mark.parametrize("which,iters", [("q0", 740), ("qe", 736)])
def test_oracle_reproduces_reference_kats(kat, which, iters):
    # KAT-1 / KAT-2: computeqgrasppose(robot, zeros, cube, CUBE_PLACEMENT[_TARGET])
    place = kat["cube_placement"] if which == "q0" else kat["cube_placement_target"]
    R, t = _placement(place)
    q, ok, it, (nl, nr) = o.computeqgrasppose(np.array(kat["seed_q"]), R, t)
    gold = np.array(kat[which])
    assert ok
    assert it == iters == kat["iters_chart"][which]
    assert np.abs(q - gold).max() <= 1e-12
    assert nl < o.EPSILON and nr < o.EPSILON


def test_joint_order_matches_notebook(kat):
    assert [j[0] for j in o.JOINTS] == kat["joint_names"]


def test_fk_at_neutral_matches_notebook(kat):
    oMl, _ = o.fk_hands(np.zeros(15))
    ref = kat["fk_q0_larm_eff"]
    assert np.abs(oMl[1] - np.array(ref["p"])).max() < 1e-12
    # printed with 6 significant digits
    assert np.abs(oMl[0] - np.array(ref["R"])).max() < 1e-6


def test_log6_roundtrip_small_and_near_pi():
    # log6 of a pure rotation about z by theta returns [0,0,0, 0,0,theta]
    for th in (1e-6, 1e-3, 0.5, 3.0, np.pi - 1e-3):
        c, s = np.cos(th), np.sin(th)
        R = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]])
        e = o.log6((R, np.zeros(3)))
        assert np.allclose(e, [0, 0, 0, 0, 0, th], atol=1e-9)


def test_fixture_cases_reproduce(oracle_cases):
    # spot-check that the committed fixtures are what the oracle computes
    for i in (2, 60):
        tg, q0 = oracle_cases["targets"][i], oracle_cases["q0"][i]
        q, ok, it, (nl, nr) = o.computeqgrasppose(q0, tg[:9].reshape(3, 3), tg[9:])
        assert ok == bool(oracle_cases["converged"][i])
        assert it == int(oracle_cases["iters"][i])
        assert np.array_equal(q, oracle_cases["q"][i])
