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

    @staticmethod
    def Interpolate(A, B, alpha: float) -> "SE3":
        """pin.SE3.Interpolate"""
        return interpolate(A, B, alpha)

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


def _skew(w):
    return np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])


_PREC3 = np.finfo(np.float64).eps ** 0.25  # Pinocchio TaylorSeriesExpansion::precision<3>()


def log6(M) -> np.ndarray:
    """pin.log6 -> [v; w] (host-side, for placement interpolation; the IK's
    log6 runs in the kernel)."""
    R, p = as_rt(M)
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    theta = 0.0 if tr > 3.0 else (math.pi if tr < -1.0 else math.acos((tr - 1.0) / 2.0))
    if theta >= math.pi - 1e-2:
        cphi = math.cos(theta - math.pi)
        beta = theta * theta / (1.0 + cphi)
        tmp = (np.diag(R) + cphi) * beta
        sgn = np.where([R[2, 1] > R[1, 2], R[0, 2] > R[2, 0], R[1, 0] > R[0, 1]], 1.0, -1.0)
        w = sgn * np.sqrt(np.maximum(tmp, 0.0))
    else:
        f = theta / math.sin(theta) if theta > _PREC3 else 1.0
        w = 0.5 * f * np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    t2 = theta * theta
    if theta < _PREC3:
        alpha, beta = 1.0 - t2 / 12.0 - t2 * t2 / 720.0, 1.0 / 12.0 + t2 / 720.0
    else:
        st, ct = math.sin(theta), math.cos(theta)
        alpha = theta * st / (2.0 * (1.0 - ct))
        beta = 1.0 / t2 - st / (2.0 * theta * (1.0 - ct))
    v = alpha * p - 0.5 * np.cross(w, p) + (beta * np.dot(w, p)) * w
    return np.concatenate([v, w])


def exp6(v) -> "SE3":
    """pin.exp6 of [v; w]."""
    lin, w = np.asarray(v[:3], dtype=np.float64), np.asarray(v[3:], dtype=np.float64)
    t2 = float(w @ w)
    t = math.sqrt(t2)
    if t < _PREC3:
        a, b, c = 1.0 - t2 / 6.0, 0.5 - t2 / 24.0, 1.0 / 6.0 - t2 / 120.0
    else:
        st, ct = math.sin(t), math.cos(t)
        a, b, c = st / t, (1.0 - ct) / t2, (t - st) / (t2 * t)
    W = _skew(w)
    WW = W @ W
    return SE3(np.eye(3) + a * W + b * WW, (np.eye(3) + b * W + c * WW) @ lin)


def interpolate(A, B, alpha: float) -> "SE3":
    """pin.SE3.Interpolate(A, B, alpha) = A * exp6(alpha * log6(A^-1 B))
    (path.py:141)."""
    Ra, ta = as_rt(A)
    Rb, tb = as_rt(B)
    a = SE3(Ra, ta)
    return a * exp6(alpha * log6(a.inverse() * SE3(Rb, tb)))


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
