"""ikgrasp — MI355X-native batched dual-arm grasp-pose IK.

Drop-in for the reference's `inverse_geometry.computeqgrasppose`
(/root/reference/inverse_geometry.py:17-100); compute runs in the HIP
library `_native/libikgrasp.so` (C-ABI: include/ikgrasp.h).
"""
from .inverse_geometry import computeqgrasppose, computeqgrasppose_batch, computeqgrasppose_multistart  # noqa: F401
from .model import DualArmModel, load_nextage, parse_urdf  # noqa: F401
from .scene import setuppinocchio, setupik  # noqa: F401
from .se3 import SE3  # noqa: F401

__version__ = "0.1.0"
