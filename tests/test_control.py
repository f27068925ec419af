"""Controller row on the CPU: the control oracle against
its committed fixtures and the identities that define the quantities
(Pinocchio's own unit tests assert the same ones), plus argument checks of
the C-ABI entry (no compute: there is no GPU here)."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLDEN
from ikgrasp import _lib
from ikgrasp.model import load_nextage
from oracle import control_oracle as co
from oracle import ik_oracle as ik


@pytest.fixture(scope="module")
def cc():
    return dict(np.load(os.path.join(GOLDEN, "control_cases.npz")))


def test_oracle_reproduces_fixtures(cc):
    for i in range(0, len(cc["q"]), 7):
        for rf in (0, 1, 2):
            r = co.frame_kinematics(cc["q"][i], cc["v"][i], rf, cc["q_des"][i], cc["v_des"][i])
            for k in ("placement", "velocity", "J", "dJ", "dJv"):
                np.testing.assert_allclose(r[k], cc[f"{k}_rf{rf}"][i], rtol=0, atol=1e-14)
        np.testing.assert_allclose(r["err"], cc["err"][i], rtol=0, atol=1e-14)
        np.testing.assert_allclose(r["derr"], cc["derr"][i], rtol=0, atol=1e-14)


def test_placement_pinned_to_ik_oracle(cc):
    """Frame placements equal the IK oracle's FK (pinned by the reference KATs)."""
    for i in range(0, len(cc["q"]), 5):
        L, R = ik.fk_hands(cc["q"][i])
        for h, (Rh, th) in enumerate((L, R)):
            np.testing.assert_allclose(cc["placement_rf2"][i, h], np.concatenate([Rh.reshape(9), th]), atol=1e-15)


@pytest.mark.parametrize("rf", [0, 1, 2])
def test_velocity_is_J_v_and_dJ_is_dJ_dt(cc, rf):
    """J v = frame velocity; dJ = d/dt J(q + t v) (central differences)."""
    h = 1e-6
    for i in range(0, len(cc["q"]), 9):
        q, v = cc["q"][i], cc["v"][i]
        J, dJ, vel = cc[f"J_rf{rf}"][i], cc[f"dJ_rf{rf}"][i], cc[f"velocity_rf{rf}"][i]
        np.testing.assert_allclose((J @ v).reshape(2, 6), vel, atol=1e-13)
        fd = (co.frame_kinematics(q + h * v, v, rf)["J"] - co.frame_kinematics(q - h * v, v, rf)["J"]) / (2 * h)
        np.testing.assert_allclose(dJ, fd, atol=5e-8 * max(1.0, np.abs(v).max()))


def test_local_jacobian_equals_ik_oracle(cc):
    """LOCAL frame Jacobian = the IK loop's computeFrameJacobian (inverse_geometry.py:75-76)."""
    for i in range(0, len(cc["q"]), 11):
        J = cc["J_rf1"][i]
        np.testing.assert_allclose(J[:6], ik.frame_jacobian_local(cc["q"][i], ik.FRAME_LEFT), atol=1e-15)
        np.testing.assert_allclose(J[6:], ik.frame_jacobian_local(cc["q"][i], ik.FRAME_RIGHT), atol=1e-15)


def test_errors_follow_control_law(cc):
    """e = [x_des - x; log3(R_des R^T)], e_dot = v_des - v (control.py:325-337)."""
    for i in range(0, len(cc["q"]), 13):
        P, Pd = cc["placement_rf2"][i], None
        rd = co.frame_kinematics(cc["q_des"][i], cc["v_des"][i], 2)
        for h in range(2):
            R, t = P[h, :9].reshape(3, 3), P[h, 9:]
            Rd, td = rd["placement"][h, :9].reshape(3, 3), rd["placement"][h, 9:]
            np.testing.assert_allclose(cc["err"][i, 6 * h:6 * h + 3], td - t, atol=1e-15)
            np.testing.assert_allclose(cc["err"][i, 6 * h + 3:6 * h + 6], ik.log3(Rd @ R.T)[0], atol=1e-15)
            np.testing.assert_allclose(cc["derr"][i, 6 * h:6 * h + 6],
                                       rd["velocity"][h] - cc["velocity_rf2"][i, h], atol=1e-15)


def test_frame_kinematics_rejects_bad_arguments():
    lib = _lib.load()
    d = _lib.model_desc(load_nextage())
    h = C.c_void_p()
    assert lib.ikg_model_create(C.byref(d), C.byref(h)) == 0
    buf = (C.c_double * 64)()
    out = _lib.FrameKinOut()
    rc = lib.ikg_frame_kinematics_batch(h, 0, 0, buf, None, None, None, 1, 7, C.byref(out), None, 0)
    assert rc == -1 and "rf" in lib.ikg_last_error().decode()
    out.err = C.cast(buf, C.c_void_p)
    rc = lib.ikg_frame_kinematics_batch(h, 0, 0, buf, None, None, None, 1, 2, C.byref(out), None, 0)
    assert rc == -1 and "q_des" in lib.ikg_last_error().decode()
    rc = lib.ikg_frame_kinematics_batch(h, 0, 0, None, None, None, None, 1, 2, C.byref(_lib.FrameKinOut()), None, 0)
    assert rc == -1 and "q is required" in lib.ikg_last_error().decode()
    rc = lib.ikg_frame_kinematics_batch(h, 0, 0, buf, None, None, None, 1, 2, None, None, 0)
    assert rc == -1 and "out is NULL" in lib.ikg_last_error().decode()
    lib.ikg_model_destroy(h)
