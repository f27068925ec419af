"""Drop-in `computeqgrasppose` (reference inverse_geometry.py:17-100) backed
by the batched HIP kernel, plus the batched / multi-start APIs.

    q, success = computeqgrasppose(robot, qcurrent, cube, cubetarget, viz=None)

Same name, positional order and return as the reference.  Differences that
a caller can observe:
  * none in `success`: when the robot carries a collision scene (the default
    from setuppinocchio) the stop test is :70's `errors pass and not
    collision(q)`, iterating on while converged-but-colliding, and a final
    colliding q is a failure (:97-98) — all inside the GPU continuation kernel;
    with `scene=None` success is the convergence test only;
  * `viz` is updated once with the final q instead of every iteration.
`qcurrent` is copied, never mutated (:49); the cube is left placed at
`cubetarget` (:42, tools.py:62-68).
"""
from __future__ import annotations

import numpy as np

from .config import CUBE_PLACEMENT, CUBE_PLACEMENT_TARGET, EPSILON, DT_IK, MAX_ITERS  # noqa: F401
from .pinocchio_bridge import is_pinocchio_like, solver_for
from .se3 import as_rt, pack_targets
from .tools import setcubeplacement


def _solver_of(robot, cube=None):
    """ikgrasp's own Robot carries its solver; a Pinocchio RobotWrapper (or
    any object with its attribute surface) gets one built from its model,
    the cube's hook frames and its collision model (pinocchio_bridge)."""
    solver = getattr(robot, "solver", None)
    if solver is not None:
        return solver
    if is_pinocchio_like(robot):
        return solver_for(robot, cube, device=getattr(robot, "device", 0))
    raise TypeError(f"robot of type {type(robot).__name__} carries no ikgrasp solver and no Pinocchio-style "
                    "model; build it with ikgrasp.scene.setuppinocchio()")


def computeqgrasppose(robot, qcurrent, cube, cubetarget, viz=None):
    """inverse_geometry.py:17 — returns (q float64[nq], success bool)."""
    setcubeplacement(robot, cube, cubetarget)  # :42
    R, t = as_rt(cubetarget)
    target = np.concatenate([R.reshape(9), t])[None, :]
    q0 = np.array(qcurrent, dtype=np.float64).copy()  # :49
    solver = _solver_of(robot, cube)
    sol = solver.solve(target, q0, dtype="f64", eps=EPSILON, dt=DT_IK, max_iters=MAX_ITERS,
                       check_collision=solver.scene is not None)
    q = sol.q[0].astype(np.float64)
    if viz is not None and hasattr(viz, "display"):  # :92-94, once with the final q
        viz.display(q)
    return q, bool(sol.converged[0])


def computeqgrasppose_batch(robot, qcurrent, cubetargets, dtype="f64", cube=None, **kw):
    """Batched API: cubetargets [B,12] / [B,4,4] / list of SE3; qcurrent [nq]
    (broadcast) or [B,nq] -> (q [B,nq], success [B], iters [B]).  `success`
    includes the collision term when the robot has a scene (override with
    check_collision=False).  `cube`: needed once for a Pinocchio-style robot."""
    targets = pack_targets(cubetargets)
    solver = _solver_of(robot, cube)
    kw.setdefault("check_collision", solver.scene is not None)
    sol = solver.solve(targets, np.asarray(qcurrent), dtype=dtype, **kw)
    return sol.q, sol.converged, sol.iters


def computeqgrasppose_multistart(robot, seeds, cubetargets, dtype="f64", cube=None, **kw):
    """Multi-start API: seeds [S,nq] x targets -> best seed per target:
    (q [T,nq], success [T], best_seed [T])."""
    targets = pack_targets(cubetargets)
    solver = _solver_of(robot, cube)
    kw.setdefault("check_collision", solver.scene is not None)
    sol = solver.solve_multistart(targets, np.asarray(seeds), dtype=dtype, **kw)
    return sol.q, sol.converged, sol.best_seed
