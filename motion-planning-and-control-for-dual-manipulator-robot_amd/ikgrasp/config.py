"""Constants of the reference scene (config.py) — same names and values.

GUI flags (config.py:15-19) and mesh paths are out of scope.
"""
import numpy as np

from .se3 import SE3, rotate

DT = 1e-3  # simulation tick time (config.py:21); the IK step is DT_IK below
EPSILON = 1e-3  # config.py:22

LEFT_HAND = "LARM_EFF"  # config.py:25
RIGHT_HAND = "RARM_EFF"
LEFT_HOOK = "LARM_HOOK"  # config.py:28
RIGHT_HOOK = "RARM_HOOK"

# scene placements (config.py:32-37)
ROBOT_PLACEMENT = SE3(np.eye(3), np.array([0.0, 0.0, 0.85]))
TABLE_PLACEMENT = SE3(rotate("z", -np.pi / 2), np.array([0.8, 0.0, 0.0]))
OBSTACLE_PLACEMENT = SE3(rotate("z", 0), np.array([0.43, -0.1, 0.94]))
CUBE_PLACEMENT = SE3(rotate("z", 0.0), np.array([0.33, -0.3, 0.93]))
CUBE_PLACEMENT_TARGET = SE3(rotate("z", 0), np.array([0.4, 0.11, 0.93]))

# IK loop hyper-parameters hard-coded in inverse_geometry.py:53-54
MAX_ITERS = 1000
DT_IK = 1e-2
