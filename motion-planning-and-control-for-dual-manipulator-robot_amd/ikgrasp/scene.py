"""Scene objects standing in for the reference's Pinocchio RobotWrappers
(setup_pinocchio.py:73-83 `setuppinocchio`).

`robot` exposes what the IK path reads from a RobotWrapper: `model.nq`,
`model.lowerPositionLimit`, `model.upperPositionLimit`, `model.names`,
`q0` (neutral = zeros, the seed used at control.py:435 and path.py:57), plus
the compiled dual-arm tables and a lazily created native solver.  `cube`
carries its placement and hook frames (cube_small.urdf:34-47).
"""
from __future__ import annotations

import numpy as np

from .config import CUBE_PLACEMENT
from .model import DualArmModel, load_nextage
from .se3 import SE3


class _ModelView:
    def __init__(self, m: DualArmModel):
        self.nq = m.nq
        self.nv = m.nq
        self.lowerPositionLimit = m.lower.copy()
        self.upperPositionLimit = m.upper.copy()
        self.names = ["universe"] + list(m.joint_names)


class Robot:
    def __init__(self, model: DualArmModel | None = None, device: int = 0, scene="nextage"):
        """scene: a CollisionScene, "nextage" (the reference scene compiled by
        tools/compile_model.py, only valid with the default model) or None."""
        self.ik_model = model if model is not None else load_nextage()
        self.model = _ModelView(self.ik_model)
        self.q0 = np.zeros(self.model.nq)
        self.device = device
        self.cube_placement = None
        self.cube_default = CUBE_PLACEMENT  # the cube geometry's placement before any setcubeplacement
        if isinstance(scene, str):
            if model is not None:
                raise ValueError("pass the CollisionScene of a custom model explicitly (or scene=None)")
            from .collision import load_nextage_scene
            scene = load_nextage_scene()
        self.scene = scene
        self._solver = None

    @property
    def solver(self):
        if self._solver is None:
            from .solver import IKSolver
            self._solver = IKSolver(self.ik_model, device=self.device, scene=self.scene)
        return self._solver


class Cube:
    def __init__(self, model: DualArmModel, placement: SE3 = CUBE_PLACEMENT):
        self._hooks = {name: SE3(model.hook_R[i], model.hook_t[i]) for i, name in enumerate(model.hook_names)}
        self.placement = placement.copy() if hasattr(placement, "copy") else placement
        self.q0 = np.zeros(0)

    def hook(self, name: str) -> SE3:
        return self._hooks[name]


def setuppinocchio(device: int = 0):
    """Same return shape as setup_pinocchio.setuppinocchio: (robot, table,
    obstacle, cube).  table/obstacle are the scene's geometry records (their
    collision geometry lives in robot.scene, as in the reference where
    loadobject appends them to the robot's collision model)."""
    robot = Robot(device=device)
    cube = Cube(robot.ik_model)
    table = next((g for g in robot.scene.geoms if g.name.startswith("baseLink")), None)
    obstacle = next((g for g in robot.scene.geoms if g.name.startswith("obstaclebase")), None)
    return robot, table, obstacle, cube


def setupik(device: int = 0):
    """Convenience: (robot, cube)."""
    robot, _, _, cube = setuppinocchio(device)
    return robot, cube
