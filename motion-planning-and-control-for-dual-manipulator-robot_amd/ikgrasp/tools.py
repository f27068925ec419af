"""Mirror of the reference helpers on the IK path (tools.py).

Same names and argument meaning.  `collision` runs the HIP collision kernel
(ikg_collision_batch) on the robot's scene with the cube at its current
placement; `distanceToObstacle` runs the HIP distance kernel
(ikg_distance_batch) over the same pairs as the reference.
"""
from __future__ import annotations

import numpy as np

from .pinocchio_bridge import is_pinocchio_like, solver_for, target_placement
from .se3 import SE3, as_rt


def jointlimitscost(robot, q):
    """tools.py:10-13"""
    up = max(q - robot.model.upperPositionLimit)
    down = max(robot.model.lowerPositionLimit - q)
    return max(0, max(up, down))


def jointlimitsviolated(robot, q):
    """tools.py:15-17"""
    return jointlimitscost(robot, q) > 0.0


def projecttojointlimits(robot, q):
    """tools.py:21-22 — np.minimum(np.maximum(lower, q), upper)."""
    return np.minimum(np.maximum(robot.model.lowerPositionLimit, q), robot.model.upperPositionLimit)


def getcubeplacement(cube, hookname=None):
    """tools.py:54-59 — oMcube (* oMf[hook] when a hook name is given).
    Like the reference, the stored cube placement is not modified."""
    R, t = as_rt(cube.placement)
    oMf = SE3(R, t)
    if hookname is not None:
        oMf = oMf * cube.hook(hookname)
    return oMf


def setcubeplacement(robot, cube, oMf):
    """tools.py:62-68 — place the cube (and the robot's copy of its collision
    geometry) at oMf.  Callers rely on this side effect (path.py:61).  A
    Pinocchio RobotWrapper gets the reference's assignments (the last robot
    geometry, the cube's geometry; the cube's updateGeometryPlacements, a
    Pinocchio call, is not repeated)."""
    if not hasattr(robot, "solver") and is_pinocchio_like(robot):
        for model, idx in ((getattr(robot, "visual_model", None), -1), (getattr(robot, "collision_model", None), -1),
                           (getattr(cube, "visual_model", None), -1), (getattr(cube, "collision_model", None), 0)):
            if model is not None:
                model.geometryObjects[idx].placement = oMf
        return
    R, t = as_rt(oMf)
    cube.placement = SE3(R, t)
    robot.cube_placement = cube.placement


def collision(robot, q):
    """tools.py:25-35 — True if any active pair of the scene intersects at q
    (the cube geometry sits where setcubeplacement last put it)."""
    solver, _ = _scene_of(robot)
    target = _cube_target(robot)
    return bool(solver.collision(np.asarray(q, dtype=np.float64).reshape(1, -1), target)[0])


def _scene_of(robot):
    solver = robot.solver if hasattr(robot, "solver") or not is_pinocchio_like(robot) else solver_for(robot)
    if solver.scene is None:
        raise RuntimeError("robot has no collision scene attached (ikgrasp.scene.setuppinocchio builds it)")
    return solver, solver.scene


def _cube_target(robot):
    if not hasattr(robot, "solver") and is_pinocchio_like(robot):
        return target_placement(robot)
    placement = robot.cube_placement if robot.cube_placement is not None else robot.cube_default
    R, t = as_rt(placement)
    return np.concatenate([R.reshape(9), t])[None, :]


def distanceToObstacle(robot, q):
    """tools.py:37-51 — shortest distance between the robot and the obstacle /
    table: min over the active pairs whose second geometry is
    'obstaclebase_0' or 'baseLink_0' of hpp-fcl's min_distance (GPU GJK)."""
    solver, scene = _scene_of(robot)
    d = solver.distance(np.asarray(q, dtype=np.float64).reshape(1, -1), _cube_target(robot), scene.obstacle_pairs())
    return float(d[0])
