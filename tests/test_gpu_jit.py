"""Model-specialised pair kernels (ikg_model_specialize, csrc/ikg_jit.hip) on the
GPU: the hipRTC-compiled loop against the same oracle fixtures and tolerances as
the prebuilt kernels, and against the prebuilt kernels themselves.

Tolerances: fp64 — identical flags and update counts, q within 1e-9 of the
oracle fixtures (1e-12 of the KATs) and within 1e-11 of the prebuilt kernel;
fp32 — hand error <= 1e-4 against the fp64 solution, counts within +-2."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from helpers import se3_err

pytestmark = pytest.mark.gpu


def _row(d):
    return np.concatenate([np.array(d["R"], dtype=np.float64).reshape(9), np.array(d["t"], dtype=np.float64)])


@pytest.fixture(scope="module")
def gc():
    return dict(np.load(os.path.join(GOLDEN, "generic_cases.npz")))


def _same(a, b, tol=1e-11):
    """Specialised vs prebuilt: identical flags and update counts; converged q
    within `tol` (folding exact 0 / 1 terms moves the last bits; the 1000-update
    unconverged runs amplify that and are compared through flags/counts only)."""
    assert np.array_equal(a.converged, b.converged) and np.array_equal(a.iters, b.iters)
    ok = b.converged
    d = float(np.abs(a.q[ok] - b.q[ok]).max()) if ok.any() else 0.0
    assert d <= tol, d


def _tilted_model():
    from ikgrasp.model import DualArmModel
    return DualArmModel.from_urdf(os.path.join(GOLDEN, "tilted_dualarm.urdf"), os.path.join(GOLDEN, "tilted_cube.urdf"))


@pytest.fixture(scope="module")
def tilted_pair():
    """(specialised, prebuilt) solvers of the tilted robot."""
    from ikgrasp.solver import IKSolver
    m = _tilted_model()
    jit, pre = IKSolver(m, device=0), IKSolver(m, device=0, specialize=False)
    jit.specialize("f64")
    jit.specialize("f32")
    yield jit, pre
    jit.close()
    pre.close()


@pytest.fixture(scope="module")
def nextage_pair():
    from ikgrasp.solver import IKSolver
    jit, pre = IKSolver(device=0), IKSolver(device=0, specialize=False)
    jit.specialize("f64")
    jit.specialize("f32")
    yield jit, pre
    jit.close()
    pre.close()


def test_specialized_flag(tilted_pair):
    jit, pre = tilted_pair
    assert jit.is_specialized("f64") and jit.is_specialized("f32")
    assert not pre.is_specialized("f64")
    jit.specialize("f64")  # idempotent


def test_auto_mode(gc):
    """Default specialize="auto": a generic model is specialised on its first
    solve per dtype; a Nextage-class model keeps the prebuilt kernels."""
    from ikgrasp.solver import IKSolver
    t, n = IKSolver(_tilted_model(), device=0), IKSolver(device=0)
    t.solve(gc["targets"][:4], gc["q0"][:4])
    n.solve(gc["targets"][:4], np.zeros(15))
    assert t.is_specialized("f64") and not t.is_specialized("f32")
    assert not n.is_specialized("f64")
    t.close()
    n.close()


def test_tilted_fp64_matches_oracle_and_prebuilt(tilted_pair, gc):
    jit, pre = tilted_pair
    a = jit.solve(gc["targets"], gc["q0"])
    b = pre.solve(gc["targets"], gc["q0"])
    ok = gc["converged"]
    assert np.array_equal(a.converged, ok) and np.array_equal(a.iters, gc["iters"])
    assert np.abs(a.q[ok] - gc["q"][ok]).max() <= 1e-9
    _same(a, b)


def test_tilted_broadcast_seed(tilted_pair, gc):
    """q0 broadcast (the non-MED loop) on the specialised kernel equals prebuilt."""
    jit, pre = tilted_pair
    a = jit.solve(gc["targets"], np.zeros(jit.nq))
    b = pre.solve(gc["targets"], np.zeros(jit.nq))
    _same(a, b)


def test_tilted_fp32_within_ee_tolerance(tilted_pair, gc):
    jit, _ = tilted_pair
    sol = jit.solve(gc["targets"], gc["q0"], dtype="f32")
    ok = gc["converged"]
    assert np.array_equal(sol.converged, ok)
    assert (np.abs(sol.iters[ok].astype(int) - gc["iters"][ok]) <= 2).all()
    h32 = jit.fk(sol.q[ok].astype(np.float64))
    h64 = jit.fk(gc["q"][ok])
    for h in range(2):
        e = se3_err(h32[:, h, :9].reshape(-1, 3, 3), h32[:, h, 9:], h64[:, h, :9].reshape(-1, 3, 3), h64[:, h, 9:])
        assert e.max() <= 1e-4


def test_tilted_damped_matches_prebuilt(tilted_pair, gc):
    jit, pre = tilted_pair
    a = jit.solve(gc["targets"], gc["q0"], lam=1e-6)
    b = pre.solve(gc["targets"], gc["q0"], lam=1e-6)
    _same(a, b)


def test_tilted_multistart(tilted_pair, gc):
    jit, _ = tilted_pair
    seeds = np.stack([np.zeros(jit.nq), gc["q_star"]])
    ms = jit.solve_multistart(gc["targets"][:8], seeds)
    for t in range(8):
        per = jit.solve(np.repeat(gc["targets"][t:t + 1], 2, axis=0), seeds)
        b = ms.best_seed[t]
        assert ms.converged[t] == per.converged[b] and np.array_equal(ms.q[t], per.q[b])


def test_nextage_kats(nextage_pair):
    jit, _ = nextage_pair
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        kat = json.load(f)
    tg = np.stack([_row(kat["cube_placement"]), _row(kat["cube_placement_target"])])
    sol = jit.solve(tg, np.zeros(15))
    assert sol.iters.tolist() == [740, 736] and sol.converged.all()
    assert np.abs(sol.q[0] - np.array(kat["q0"])).max() <= 1e-12
    assert np.abs(sol.q[1] - np.array(kat["qe"])).max() <= 1e-12


def test_nextage_fixtures_fp64(nextage_pair, oracle_cases):
    """Per-problem seeds: the specialised frame-1 loop with the medium-range series."""
    jit, pre = nextage_pair
    c = oracle_cases
    a = jit.solve(c["targets"], c["q0"])
    b = pre.solve(c["targets"], c["q0"])
    assert np.array_equal(a.converged, c["converged"]) and np.array_equal(a.iters, c["iters"])
    conv = c["converged"]
    assert np.abs(a.q[conv] - c["q"][conv]).max() <= 1e-9
    _same(a, b)


def test_nextage_fixtures_fp32(nextage_pair, oracle_cases):
    jit, _ = nextage_pair
    c = oracle_cases
    sol = jit.solve(c["targets"], c["q0"], dtype="f32", variant=1)  # PAIR: the layout the JIT replaces
    conv = c["converged"]
    assert (np.abs(sol.iters[conv].astype(int) - c["iters"][conv]) <= 2).all()
    h32 = jit.fk(sol.q[conv].astype(np.float64))
    h64 = jit.fk(c["q"][conv])
    for h in range(2):
        e = se3_err(h32[:, h, :9].reshape(-1, 3, 3), h32[:, h, 9:], h64[:, h, :9].reshape(-1, 3, 3), h64[:, h, 9:])
        assert e.max() <= 1e-4


def test_ragged_batches(tilted_pair, gc):
    jit, pre = tilted_pair
    for B in (1, 31, 33):
        a = jit.solve(gc["targets"][:B], gc["q0"][:B])
        b = pre.solve(gc["targets"][:B], gc["q0"][:B])
        _same(a, b)


def _tilted_scene(model):
    """The tilted robot's URDF collision primitives plus a world-fixed table box
    and the grasp cube (a 0.1 m box at each solve's target); every pair of
    geometries on different joints."""
    import xml.etree.ElementTree as ET

    from ikgrasp.collision import BOX, CollisionScene, Geom, _link_geoms, _robot_link_frames
    root = ET.parse(os.path.join(GOLDEN, "tilted_dualarm.urdf")).getroot()
    geoms = _link_geoms(root, _robot_link_frames(root, model.joint_names, model.axis_frames()))
    geoms.append(Geom("table_0", BOX, -1, "table", np.eye(3), np.array([0.6, 0.0, 0.55]),
                      np.array([0.3, 0.6, 0.05])))
    geoms.append(Geom("cube_0", BOX, -1, "cube", np.eye(3), np.zeros(3), np.array([0.05, 0.05, 0.05]), True))
    n = len(geoms)
    pairs = [(i, j) for i in range(n) for j in range(i + 1, n) if geoms[i].joint != geoms[j].joint]
    return CollisionScene(geoms, np.array(pairs, dtype=np.int32))


def test_tilted_collision_term_specialised_vs_prebuilt(gc):
    """check_collision on a generic model: the specialised batch kernel followed
    by the (prebuilt, generic-table) collision continuation gives the prebuilt
    path's flags and update counts; successful solves are collision-free."""
    from ikgrasp.solver import IKSolver
    m = _tilted_model()
    scene = _tilted_scene(m)
    jit, pre = IKSolver(m, device=0, scene=scene), IKSolver(m, device=0, scene=scene, specialize=False)
    a = jit.solve(gc["targets"], gc["q0"], check_collision=True)
    assert jit.is_specialized("f64")
    b = pre.solve(gc["targets"], gc["q0"], check_collision=True)
    _same(a, b, tol=1e-9)
    ok = a.converged.astype(bool)
    assert ok.any()
    assert not jit.collision(a.q[ok], gc["targets"][ok]).any()
    jit.close()
    pre.close()
