"""Minimal SE(3) value type with the attribute surface the reference uses on
`pinocchio.SE3` (`.rotation`, `.translation`, `*`, `.inverse()`,
`.homogeneous`).  Anything exposing `.rotation`/`.translation` (a real
`pin.SE3`) or a 4x4 array is accepted wherever a placement is expected.
"""
from __future__ import annotations

import math

import numpy as np


class SE3:
    __slots__ = ("rotation", "translation")

    def __init__(self, rotation=None, translation=None):
        self.rotation = np.eye(3) if rotation is None else np.array(rotation, dtype=np.float64).reshape(3, 3)
        self.translation = np.zeros(3) if translation is None else np.array(translation, dtype=np.float64).reshape(3)

    @staticmethod
    def Identity() -> "SE3":
        return SE3()

    def __mul__(self, other: "SE3") -> "SE3":
        return SE3(self.rotation @ other.rotation, self.translation + self.rotation @ other.translation)

    def inverse(self) -> "SE3":
        Rt = self.rotation.T
        return SE3(Rt, -(Rt @ self.translation))

    @property
    def homogeneous(self) -> np.ndarray:
        H = np.eye(4)
        H[:3, :3] = self.rotation
        H[:3, 3] = self.translation
        return H

    def copy(self) -> "SE3":
        return SE3(self.rotation.copy(), self.translation.copy())

    def __repr__(self) -> str:
        return f"SE3(R={self.rotation.tolist()}, p={self.translation.tolist()})"


def rotate(axis: str, angle: float) -> np.ndarray:
    """pinocchio.utils.rotate (used by config.py:34-37)."""
    c, s = math.cos(angle), math.sin(angle)
    if axis == "x":
        return np.array([[1.0, 0.0, 0.0], [0.0, c, -s], [0.0, s, c]])
    if axis == "y":
        return np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])
    if axis == "z":
        return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])
    raise ValueError(f"unknown axis {axis!r}")


def as_rt(placement):
    """(R[3,3], t[3]) float64 from an SE3-like object, a 4x4 or a flat 12-vector
    (R row-major then t, the C-ABI target layout)."""
    if hasattr(placement, "rotation") and hasattr(placement, "translation"):
        return (np.asarray(placement.rotation, dtype=np.float64).reshape(3, 3),
                np.asarray(placement.translation, dtype=np.float64).reshape(3))
    a = np.asarray(placement, dtype=np.float64)
    if a.shape == (4, 4):
        return a[:3, :3].copy(), a[:3, 3].copy()
    if a.shape == (12,):
        return a[:9].reshape(3, 3).copy(), a[9:].copy()
    raise TypeError(f"cannot interpret {type(placement).__name__} of shape {getattr(a, 'shape', None)} as a placement")


def pack_targets(placements) -> np.ndarray:
    """Stack placements into the C-ABI layout [B, 12] = (R row-major, t)."""
    if isinstance(placements, np.ndarray) and placements.ndim == 2 and placements.shape[1] == 12:
        return np.ascontiguousarray(placements, dtype=np.float64)
    if isinstance(placements, np.ndarray) and placements.ndim == 3 and placements.shape[1:] == (4, 4):
        out = np.empty((placements.shape[0], 12))
        out[:, :9] = placements[:, :3, :3].reshape(-1, 9)
        out[:, 9:] = placements[:, :3, 3]
        return out
    rows = []
    for p in placements:
        R, t = as_rt(p)
        rows.append(np.concatenate([R.reshape(9), t]))
    return np.array(rows, dtype=np.float64).reshape(-1, 12)
