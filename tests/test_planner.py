"""Planner row on the CPU: the oracle's distance methods agree
with each other, the golden fixtures match the product's scene, the host-side
SE3.Interpolate matches the oracle, and the batched sampler's RandomState
arithmetic is the reference's (path.py:41-43)."""
import os
import warnings

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import collision_oracle as co
from oracle import planner_oracle as po


@pytest.fixture(scope="module")
def planner_cases():
    return dict(np.load(os.path.join(GOLDEN, "planner_cases.npz")))


@pytest.fixture(scope="module")
def oscene():
    return co.load_scene(os.path.join(GOLDEN, "collision_scene.json"))


def _rot(seed):
    from scipy.spatial.transform import Rotation
    return Rotation.random(random_state=seed).as_matrix()


def test_box_box_distance_lsq_matches_convex_program():
    rng = np.random.default_rng(0)
    warnings.filterwarnings("ignore")
    for i in range(12):
        ga = {"kind": po.BOX, "dims": rng.uniform(0.02, 0.2, 3)}
        gb = {"kind": po.BOX, "dims": rng.uniform(0.02, 0.2, 3)}
        Ra, Rb, ta, tb = _rot(i), _rot(50 + i), rng.normal(size=3) * 0.3, rng.normal(size=3) * 0.3
        d1 = po._box_box_distance(Ra, ta, ga["dims"], Rb, tb, gb["dims"])
        d2 = po._slsqp_distance(ga, Ra, ta, gb, Rb, tb)
        assert abs(d1 - d2) <= 1e-9


def test_sphere_box_distance_exact_matches_convex_program():
    rng = np.random.default_rng(1)
    warnings.filterwarnings("ignore")
    for i in range(12):
        gs = {"kind": po.SPHERE, "dims": np.array([rng.uniform(0.02, 0.1), 0.0, 0.0])}
        gb = {"kind": po.BOX, "dims": rng.uniform(0.02, 0.2, 3)}
        Rb, ts, tb = _rot(i), rng.normal(size=3) * 0.3, rng.normal(size=3) * 0.3
        d1 = po.pair_distance(gs, np.eye(3), ts, gb, Rb, tb)
        d2 = po._slsqp_distance(gs, np.eye(3), ts, gb, Rb, tb) - gs["dims"][0]
        assert abs(d1 - d2) <= 1e-9


def test_fixture_pairs_are_the_products_obstacle_pairs(planner_cases, oscene):
    from ikgrasp.collision import load_nextage_scene
    sc = load_nextage_scene()
    assert np.array_equal(planner_cases["pair_idx"], sc.obstacle_pairs())
    assert np.array_equal(planner_cases["pair_idx"], np.array(po.obstacle_pairs(oscene)))
    assert list(sc.env_geoms()) == list(po.env_ids(oscene))
    assert len(planner_cases["pair_idx"]) == 78  # 39 moving robot geometries x {table, obstacle}


def test_host_interpolate_matches_oracle():
    from ikgrasp import se3
    for i in range(6):
        A = se3.SE3(_rot(i), [0.1 * i, 0.2, 0.3])
        B = se3.SE3(_rot(10 + i), [0.4, -0.2, 1.0 - 0.1 * i])
        for a in (0.0, 0.25, 0.5, 1.0):
            C = se3.SE3.Interpolate(A, B, a)
            R, t = po.se3_interpolate((A.rotation, A.translation), (B.rotation, B.translation), a)
            assert np.abs(C.rotation - R).max() <= 1e-14 and np.abs(C.translation - t).max() <= 1e-14
    # pure translations (the planner's placements): exact lerp
    A, B = se3.SE3(np.eye(3), [0.33, -0.3, 0.93]), se3.SE3(np.eye(3), [0.4, 0.11, 1.2])
    C = se3.interpolate(A, B, 0.3)
    assert np.array_equal(C.rotation, np.eye(3))
    assert np.abs(C.translation - (A.translation + 0.3 * (B.translation - A.translation))).max() <= 1e-16


def test_batched_draws_reproduce_randomstate_uniform():
    lo, hi = np.array([0.33, -0.3, 1.05]), np.array([0.4, 0.11, 1.4])
    np.random.seed(5)
    seq = np.array([[np.random.uniform(lo[k], hi[k]) for k in range(3)] for _ in range(40)])
    after_seq = np.random.random_sample()
    np.random.seed(5)
    batch = lo + (hi - lo) * np.random.random_sample((40, 3))
    assert np.array_equal(seq, batch)
    np.random.seed(5)
    np.random.random_sample(3 * 40)
    assert np.random.random_sample() == after_seq


def test_planner_fixture_consistency(planner_cases, oscene):
    c = planner_cases
    # each sample reproduces from its seed with the reference's draw order
    for seed in range(len(c["sample_t"])):
        rs = np.random.RandomState(seed)
        draws = []
        for _ in range(int(c["sample_attempts"][seed])):
            draws.append([rs.uniform(0.33, 0.4), rs.uniform(-0.3, 0.11), rs.uniform(1.05, 1.4)])
        assert np.array_equal(np.array(draws[-1]), c["sample_t"][seed])
        assert rs.random_sample() == c["sample_next"][seed]
    # the minimum over pairs is what distanceToObstacle returns
    assert c["dist"].shape == (len(c["dist_q"]), len(c["pair_idx"]))
    assert c["path_q"].shape[0] == c["path_t"].shape[0] >= 2 and c["pathb_q"].shape[0] == 1
