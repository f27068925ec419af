"""CPU ORACLE — test infrastructure only, never the product path.

numpy restatement of the controller's kinematic terms (SURVEY.md §8 row f-4,
`/root/reference/control.py:284-345`) in Pinocchio's own formulation, i.e. by
spatial algebra over the joint tree rather than by the point-velocity
formulas the HIP kernel uses (csrc/ikg_control.hip), so the two are
independent derivations:

  pin.forwardKinematics(model, data, q, v)      v_i = liMi.actInv(v_parent) + S_i v_i,  ov_i = oMi.act(v_i)
  pin.computeJointJacobiansTimeVariation        J_i = oMi.act(S_i),  dJ_i = ov_i x J_i   (motion cross product)
  pin.getFrameJacobian(..., rf)                 WORLD: J_i;  LOCAL_WORLD_ALIGNED: linear -= p_f x angular;
                                                LOCAL: oMf.actInv(J_i)
  pin.getFrameJacobianTimeVariation(..., rf)    WORLD: dJ_i;
                                                LOCAL_WORLD_ALIGNED: shift dJ_i to p_f, then
                                                  linear -= (ov_joint.linear + ov_joint.angular x p_f) x J_i.angular;
                                                LOCAL: oMf.actInv(dJ_i) - v_f x oMf.actInv(J_i)
  pin.getFrameVelocity(..., rf)                 v_f = fMi.actInv(v_joint), expressed in rf
  control.py:325-337                            e = [x_des - x; log3(R_des R^T)], e_dot = v_des - v (LWA)

Parity status: the FK and frame placement are pinned by the IK oracle's KATs
(`ik_oracle`, lab_instructions.ipynb:290-293 and trajectory.json).  The
velocity / Jacobian-time-variation semantics are Pinocchio's (third-party,
not in the reference tree, no golden outputs there): this file is checked by
the defining identities instead — J v equals the frame velocity, and dJ
equals the finite-difference derivative of J along v in every rf, which is
the property Pinocchio's own unit tests assert for
getFrameJacobianTimeVariation — so against Pinocchio's outputs parity is
UNPINNED beyond those identities.
"""
from __future__ import annotations

import numpy as np

from oracle import ik_oracle as ik

WORLD, LOCAL, LOCAL_WORLD_ALIGNED = 0, 1, 2
FRAMES = (ik.FRAME_LEFT, ik.FRAME_RIGHT)


def _S(j):
    s = np.zeros(6)
    s[3 + ik.AXIS[j]] = 1.0  # revolute: [0; axis]
    return s


def act(M, m):
    """SE3.act on a motion [linear; angular]."""
    R, p = M
    w = R @ m[3:]
    return np.concatenate([R @ m[:3] + np.cross(p, w), w])


def act_inv(M, m):
    """SE3.actInv on a motion."""
    R, p = M
    return np.concatenate([R.T @ (m[:3] - np.cross(p, m[3:])), R.T @ m[3:]])


def motion_cross(a, b):
    """Motion x motion: [w_a x v_b + v_a x w_b; w_a x w_b]."""
    return np.concatenate([np.cross(a[3:], b[:3]) + np.cross(a[:3], b[3:]), np.cross(a[3:], b[3:])])


def forward_kinematics_v(q, v):
    """pin.forwardKinematics(model, data, q, v): oMi, local v_i, world ov_i."""
    placements = ik.joint_placements()
    oMi, vl, ov = [], [], []
    for j in range(ik.NQ):
        R0, t0 = placements[j]
        liMi = (R0 @ ik.axis_rotation(ik.AXIS[j], q[j]), t0.copy())
        vj = _S(j) * v[j]
        if ik.PARENT[j] >= 0:
            vj = vj + act_inv(liMi, vl[ik.PARENT[j]])
            M = ik.se3_mul(oMi[ik.PARENT[j]], liMi)
        else:
            M = liMi
        oMi.append(M)
        vl.append(vj)
        ov.append(act(M, vj))
    return oMi, vl, ov


def _support(j):
    out = []
    while j >= 0:
        out.append(j)
        j = ik.PARENT[j]
    return out


def frame_terms(q, v, frame, rf):
    """(oMf, v_frame [6], J [6,nq], dJ [6,nq]) of one frame in rf."""
    q = np.asarray(q, dtype=np.float64)
    v = np.asarray(v, dtype=np.float64)
    oMi, vl, ov = forward_kinematics_v(q, v)
    j, Rf, tf = frame
    fM = (Rf, tf)
    oMf = ik.se3_mul(oMi[j], fM)
    Rw, p = oMf
    J = np.zeros((6, ik.NQ))
    dJ = np.zeros((6, ik.NQ))
    v_f = act_inv(fM, vl[j])  # frame velocity, LOCAL
    for i in _support(j):
        Jw = act(oMi[i], _S(i))
        dJw = motion_cross(ov[i], Jw)  # computeJointJacobiansTimeVariation
        if rf == WORLD:
            J[:, i], dJ[:, i] = Jw, dJw
        elif rf == LOCAL_WORLD_ALIGNED:
            J[:, i] = np.concatenate([Jw[:3] - np.cross(p, Jw[3:]), Jw[3:]])
            d = np.concatenate([dJw[:3] - np.cross(p, dJw[3:]), dJw[3:]])
            d[:3] -= np.cross(ov[j][:3] + np.cross(ov[j][3:], p), Jw[3:])
            dJ[:, i] = d
        else:
            Jl = act_inv(oMf, Jw)
            J[:, i] = Jl
            dJ[:, i] = act_inv(oMf, dJw) - motion_cross(v_f, Jl)
    if rf == LOCAL:
        vel = v_f
    elif rf == LOCAL_WORLD_ALIGNED:
        vel = np.concatenate([Rw @ v_f[:3], Rw @ v_f[3:]])
    else:
        vel = act(oMf, v_f)
    return oMf, vel, J, dJ


def frame_kinematics(q, v, rf=LOCAL_WORLD_ALIGNED, q_des=None, v_des=None):
    """Both hands for one state, in the layout of ikg_frame_kinematics_batch:
    placement [2,12], velocity [2,6], J/dJ [12,nq], dJv [12] (+ err/derr [12]
    when q_des is given)."""
    out = {"placement": np.zeros((2, 12)), "velocity": np.zeros((2, 6)), "J": np.zeros((12, ik.NQ)),
           "dJ": np.zeros((12, ik.NQ)), "dJv": np.zeros(12)}
    v = np.zeros(ik.NQ) if v is None else np.asarray(v, dtype=np.float64)
    for h, frame in enumerate(FRAMES):
        (R, p), vel, J, dJ = frame_terms(q, v, frame, rf)
        out["placement"][h] = np.concatenate([R.reshape(9), p])
        out["velocity"][h] = vel
        out["J"][6 * h:6 * h + 6] = J
        out["dJ"][6 * h:6 * h + 6] = dJ
        out["dJv"][6 * h:6 * h + 6] = dJ @ v
    if q_des is not None:
        vd = np.zeros(ik.NQ) if v_des is None else np.asarray(v_des, dtype=np.float64)
        e = np.zeros(12)
        ed = np.zeros(12)
        for h, frame in enumerate(FRAMES):
            (R, p), vel, _, _ = frame_terms(q, v, frame, LOCAL_WORLD_ALIGNED)
            (Rd, pd), veld, _, _ = frame_terms(q_des, vd, frame, LOCAL_WORLD_ALIGNED)
            e[6 * h:6 * h + 3] = pd - p  # control.py:326
            e[6 * h + 3:6 * h + 6] = ik.log3(Rd @ R.T)[0]  # :327
            ed[6 * h:6 * h + 6] = veld - vel  # :330-331
        out["err"], out["derr"] = e, ed
    return out


def task_space_terms(q, vq, q_des, vq_des):
    """control.py:284-345 kinematic block -> (J_total [12,nq], J_dot_v_total
    [12], e [12], e_dot [12]) with LOCAL_WORLD_ALIGNED Jacobians."""
    r = frame_kinematics(q, vq, LOCAL_WORLD_ALIGNED, q_des, vq_des)
    return r["J"], r["dJv"], r["err"], r["derr"]
