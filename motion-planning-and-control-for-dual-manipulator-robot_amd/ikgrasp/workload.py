"""Synthetic grasp-target batches (the reference's own sampling distributions).

* `uniform_targets`: path.py:35-47 `sample_cube_placement` — cube translation
  x in [0.33, 0.40] (CUBE_PLACEMENT / _TARGET x), y in [-0.30, 0.11], z in
  [1.05, 1.40], rotation = identity.
* `yaw`: the "random SE(3)" variant adds a yaw ~ U[-pi/4, pi/4]
  (cf. the 45-degree rotated case, inverse_geometry_TESTS.py:266).
* `random_seeds`: multi-start seeds q ~ U(joint limits) with the passive
  (head) joints at 0.
Deterministic: numpy default_rng(seed).
"""
from __future__ import annotations

import numpy as np

X_RANGE = (0.33, 0.40)   # min/max of CUBE_PLACEMENT, CUBE_PLACEMENT_TARGET x (config.py:36-37)
Y_RANGE = (-0.30, 0.11)
Z_RANGE = (1.05, 1.40)   # path.py:38


def uniform_targets(n: int, seed: int = 0, yaw: float = 0.0) -> np.ndarray:
    """[n, 12] cube placements (R row-major, t)."""
    rng = np.random.default_rng(seed)
    t = np.stack([rng.uniform(*X_RANGE, n), rng.uniform(*Y_RANGE, n), rng.uniform(*Z_RANGE, n)], axis=1)
    out = np.zeros((n, 12))
    if yaw > 0:
        a = rng.uniform(-yaw, yaw, n)
        c, s = np.cos(a), np.sin(a)
        out[:, 0], out[:, 1], out[:, 3], out[:, 4], out[:, 8] = c, -s, s, c, 1.0
    else:
        out[:, 0] = out[:, 4] = out[:, 8] = 1.0
    out[:, 9:] = t
    return out


def random_seeds(model, S: int, seed: int = 0) -> np.ndarray:
    """[S, nq] joint configurations uniform within the limits, passive joints 0."""
    rng = np.random.default_rng(seed)
    q = rng.uniform(model.lower, model.upper, size=(S, model.nq))
    q[:, model.passive_q] = 0.0
    return q
