"""Controller kinematics on the GPU.

The reference controller (`/root/reference/control.py:242-410`, `controllaw`)
spends its kinematic work, per tick, in Pinocchio calls over the two hands:

    pin.computeAllTerms(model, data, q, vq); pin.updateFramePlacements      (:284-287)
    pin.computeJointJacobians / computeJointJacobiansTimeVariation          (:288-289)
    pin.forwardKinematics(model, data_des, q_des, vq_des)                   (:292-294)
    oMee = data.oMf[fid]; v_frame = pin.getFrameVelocity(..., LWA)          (:305-313)
    the same for the desired state                                          (:316-322)
    e = [x_des - x; log3(R_des R^T)], e_dot = v_des - v                     (:325-337)
    J = pin.computeFrameJacobian(..., LWA)                                   (:341-342)
    J_dot = pin.getFrameJacobianTimeVariation(..., LWA); J_dot @ vq          (:343-345)
    np.vstack / np.hstack over the two hands                                 (:368-371)

`task_space_terms` returns those stacked quantities for one state (the
drop-in for that block); `task_space_terms_batch` does many states in one
launch of `ikg_frame_kinematics_batch` (GPU).  The dynamics (M, b from
computeAllTerms / nonLinearEffects), the QP (quadprog) and the simulator stay
out of scope.  There is no CPU path: without the HIP library
these raise `NativeLibraryError`.
"""
from __future__ import annotations

import numpy as np

from . import _lib

WORLD, LOCAL, LOCAL_WORLD_ALIGNED = _lib.IKG_WORLD, _lib.IKG_LOCAL, _lib.IKG_LOCAL_WORLD_ALIGNED
HANDS = ("LARM_EFF", "RARM_EFF")  # control.py:273-276, row blocks 0-5 / 6-11


def frame_kinematics(robot, q, vq=None, rf=LOCAL_WORLD_ALIGNED, outputs=("placement", "velocity", "J", "dJ", "dJv"),
                     dtype="f64"):
    """Per-hand frame placement, velocity, Jacobian and its time variation
    in `rf` for a batch of states q, vq [B,nq] (GPU)."""
    return robot.solver.frame_kinematics(q, vq, rf=rf, outputs=outputs, dtype=dtype)


def task_space_terms_batch(robot, q, vq, q_des, vq_des, dtype="f64"):
    """control.py:284-345 for B states at once -> dict of
      J_total      [B,12,nq]  np.vstack of the hands' LOCAL_WORLD_ALIGNED Jacobians (:369)
      J_dot_v      [B,12]     J_dot @ vq per hand, stacked (:345, :370)
      e            [B,12]     [x_des - x; log3(R_des R^T)] per hand (:325-327, :335)
      e_dot        [B,12]     v_des - v per hand (:330-336)
      oMf          [B,2,12]   current hand placements (R row-major, t)
      v_frame      [B,2,6]    current hand velocities (LOCAL_WORLD_ALIGNED)."""
    r = robot.solver.frame_kinematics(q, vq, q_des, vq_des, rf=LOCAL_WORLD_ALIGNED,
                                      outputs=("placement", "velocity", "J", "dJv", "err", "derr"), dtype=dtype)
    return {"J_total": r["J"], "J_dot_v": r["dJv"], "e": r["err"], "e_dot": r["derr"], "oMf": r["placement"],
            "v_frame": r["velocity"]}


def task_space_terms(robot, q, vq, q_des, vq_des):
    """One controller tick's kinematic terms (control.py:284-345) ->
    (J_total [12,nq], J_dot_v_total [12], e [12], e_dot [12]), float64."""
    row = lambda x: np.asarray(x, dtype=np.float64).reshape(1, -1)
    r = task_space_terms_batch(robot, row(q), row(vq), row(q_des), row(vq_des))
    return r["J_total"][0], r["J_dot_v"][0], r["e"][0], r["e_dot"][0]
