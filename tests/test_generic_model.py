"""Model generality on the CPU: joint axes that are
negative or not aligned with a frame axis (Pinocchio's RevoluteUnaligned)
compiled onto canonical axes by re-expressing joint frames (ikgrasp/model.py),
checked against oracle/generic_oracle.py (raw axes, Rodrigues) on the
synthetic robot tests/golden/tilted_dualarm.urdf, and the kernel arithmetic
(host emulator, generic path) against the oracle's IK fixtures."""
import ctypes as C
import os
import xml.etree.ElementTree as ET

import numpy as np

import helpers
import pytest

from conftest import GOLDEN
from helpers import fk_tables, hands_from_tables
from ikgrasp import _lib
from ikgrasp.collision import _link_geoms, _robot_link_frames
from ikgrasp.model import DualArmModel, axis_frame, parse_urdf
from oracle import generic_oracle as go
from oracle import ik_oracle as ik

ROBOT = os.path.join(GOLDEN, "tilted_dualarm.urdf")
CUBE = os.path.join(GOLDEN, "tilted_cube.urdf")
REF = "/root/reference"


@pytest.fixture(scope="module")
def gc():
    return dict(np.load(os.path.join(GOLDEN, "generic_cases.npz")))


@pytest.fixture(scope="module")
def model():
    return DualArmModel.from_urdf(ROBOT, CUBE)


@pytest.mark.parametrize("e", [(1, 0, 0), (0, 1, 0), (0, 0, 1), (-1, 0, 0), (0, -1, 0), (0, 0, -1),
                               (0, 0.6, 0.8), (0, -0.6, 0.8), (0.48, -0.6, 0.64), (-0.8, 0.0, -0.6)])
def test_axis_frame(e):
    e = np.array(e, dtype=np.float64)
    c, Q = axis_frame(e)
    u = np.zeros(3)
    u[c] = 1.0
    np.testing.assert_allclose(Q @ u, e, atol=1e-15)
    np.testing.assert_allclose(Q.T @ Q, np.eye(3), atol=1e-15)
    assert abs(np.linalg.det(Q) - 1.0) < 1e-15 and abs(e[c]) == np.abs(e).max()
    if np.count_nonzero(e) == 1:
        assert set(np.unique(Q)) <= {-1.0, 0.0, 1.0}  # exact for signed canonical axes


def test_structure(model):
    assert model.nq == 14 and model.root_q == 0 and model.passive_q == [1]
    assert model.axis.tolist() == [2, 2, 2, 1, 1, 0, 2, 2, 2, 1, 1, 0, 2, 2]
    assert not np.allclose(model.axis_frames(), np.eye(3))  # conjugated joints exist


def test_compiled_fk_and_jacobian_match_raw_axis_oracle(model, gc):
    for q, hands, J in zip(gc["fk_q"], gc["fk_hands"], gc["fk_J"]):
        np.testing.assert_allclose(hands_from_tables(model, q), hands, atol=1e-14)
        # LOCAL frame Jacobian from the compiled tables: world axis = joint frame column
        oMi = fk_tables(model, q)
        for h in range(2):
            Rf = hands[h, :9].reshape(3, 3)
            pf = hands[h, 9:]
            Jt = np.zeros((6, model.nq))
            for j in [model.root_q] + list(model.arm_q[h]):
                a = oMi[j][0][:, int(model.axis[j])]
                Jt[:3, j] = Rf.T @ np.cross(a, pf - oMi[j][1])
                Jt[3:, j] = Rf.T @ a
            np.testing.assert_allclose(Jt, J[6 * h:6 * h + 6], atol=1e-14)


def test_collision_geometries_follow_the_conjugated_frames(model, gc):
    """Geometry placements compiled with the model's axis frames land where
    the raw-axis oracle puts them."""
    root = ET.parse(ROBOT).getroot()
    geoms = {g.name: g for g in _link_geoms(root, _robot_link_frames(root, model.joint_names, model.axis_frames()))}
    names = [str(n) for n in gc["geo_names"]]
    for q, geo in zip(gc["fk_q"][:8], gc["geo"][:8]):
        oMi = fk_tables(model, q)
        for name, ref in zip(names, geo):
            g = geoms[name]
            R, t = (g.R, g.t) if g.joint < 0 else ik.se3_mul(oMi[g.joint], (g.R, g.t))
            np.testing.assert_allclose(np.concatenate([R.reshape(9), t]), ref, atol=1e-14, err_msg=name)


@pytest.mark.parametrize("variant", [0, 99])
def test_emulated_kernel_solves_tilted_robot(model, gc, variant):
    """The kernel's device functions (host emulator, generic path: runtime
    axes, placement rotations) reproduce the raw-axis oracle: same convergence
    flags and update counts, q within 1e-9.  variant 0: the model's own
    specialisation -- the tilted robot's wrist joints meet in a point, so the
    decoupled wrist solve (SpecGenericWrist); 99: forced SpecGeneric, the 6x6
    Householder QR."""
    emu = helpers.emu_path()
    if not os.path.exists(emu):
        pytest.skip("libikgrasp_emu.so not built")
    lib = C.CDLL(emu)
    vp = C.c_void_p
    lib.ikg_emu_solve.argtypes = [vp, C.c_int, vp, vp, C.c_int64, C.c_int64, vp, vp, vp, vp, vp, vp, C.c_int, vp]
    desc = _lib.model_desc(model)
    tg, q0 = np.ascontiguousarray(gc["targets"]), np.ascontiguousarray(gc["q0"])
    B = len(tg)
    p = _lib.default_params()
    p.variant = variant
    q, conv, it, err = np.empty((B, model.nq)), np.empty(B, np.uint8), np.empty(B, np.int32), np.empty((B, 2))
    assert lib.ikg_emu_solve(C.byref(desc), 0, tg.ctypes.data, q0.ctypes.data, model.nq, B, C.byref(p),
                             q.ctypes.data, conv.ctypes.data, it.ctypes.data, err.ctypes.data, None, 0, None) == 0
    ok = gc["converged"]
    assert np.array_equal(conv.astype(bool), ok) and np.array_equal(it, gc["iters"])
    assert np.abs(q[ok] - gc["q"][ok]).max() <= 1e-9


def test_generic_oracle_reproduces_kats(kat):
    """The raw-axis restatement on the reference's own URDF gives KAT-1/2."""
    urdf = os.path.join(REF, "models/nextagea_description/urdf/NextageaOpen.urdf")
    if not os.path.exists(urdf):
        pytest.skip("reference tree not present")
    m = go.ChainModel(urdf, (np.eye(3), np.array([0.0, 0.0, 0.85])))
    hooks = go.cube_hooks(os.path.join(REF, "models/cubes/cube_small.urdf"))
    for key, qk, n in (("cube_placement", "q0", 740), ("cube_placement_target", "qe", 736)):
        q, ok, it, _ = go.computeqgrasppose(m, hooks, np.zeros(15), np.array(kat[key]["R"]), np.array(kat[key]["t"]))
        assert ok and it == n and np.abs(q - np.array(kat[qk])).max() < 1e-14


def test_unmodelled_joints_rejected():
    base = open(ROBOT).read()
    with pytest.raises(ValueError, match="zero axis"):
        parse_urdf(base.replace('<axis xyz="0 0.6 0.8"/>', '<axis xyz="0 0 0"/>'))
    with pytest.raises(ValueError, match="unsupported"):
        parse_urdf(base.replace('name="HEAD_JOINT0" type="revolute"', 'name="HEAD_JOINT0" type="prismatic"'))
