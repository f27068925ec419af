"""Planner-side callers of the IK: the reference's path.py
sampler and path projection, with every IK solve, collision check and
distance query batched on the GPU.

    q, placement = sample_cube_placement(robot, cube, cubeplacementq0, cubeplacementqgoal, viz=None)
    robot_path, cube_path = project_path(robot, cube, q_curr, cube_curr, cube_rand, step_size=0.025, viz=None)

Same names, arguments and results as /root/reference/path.py:27-62 and
:125-163.  `sample_cube_placement` draws its candidates from numpy's global
RandomState exactly as the reference does (x, y, z per attempt) but
evaluates them a batch at a time: cube-vs-environment check
(ikg_target_env_batch), cold-start IK with the collision term
(ikg_solve_batch), distanceToObstacle (ikg_distance_batch); the first valid
candidate in draw order is returned and the RandomState is left exactly
where the reference's sequential loop would leave it.  The reference's
progress prints are not reproduced; `viz` is shown once with the result.

Batched variants for planners that can use many samples / projections at
once: `sample_cube_placements` (n valid samples) and `project_paths` (many
warm-started projection chains advanced in lock-step, one batched solve per
step).
"""
from __future__ import annotations

import numpy as np

from .config import DT_IK, EPSILON, MAX_ITERS
from .se3 import SE3, as_rt, interpolate
from .tools import setcubeplacement

MIN_OBSTACLE_DISTANCE = 0.04  # path.py:32
Z_RANGE = (1.05, 1.4)  # path.py:38


def _solver_scene(robot):
    solver = robot.solver
    if solver.scene is None:
        raise RuntimeError("the planner needs the robot's collision scene (ikgrasp.scene.setuppinocchio)")
    return solver, solver.scene


def _bounds(cubeplacementq0, cubeplacementqgoal):
    _, a = as_rt(cubeplacementq0)
    _, b = as_rt(cubeplacementqgoal)
    return ((min(a[0], b[0]), max(a[0], b[0])), (min(a[1], b[1]), max(a[1], b[1])), Z_RANGE)


def _rows(points):
    """placements [B,12] with identity rotation (path.py:48)."""
    out = np.zeros((points.shape[0], 12))
    out[:, [0, 4, 8]] = 1.0
    out[:, 9:] = points
    return out


def _evaluate(robot, placements, q0):
    """Candidates -> (valid [B] bool, q [B,nq]) per path.py:51-62."""
    solver, scene = _solver_scene(robot)
    B = placements.shape[0]
    valid = np.zeros(B, dtype=bool)
    q = np.zeros((B, solver.nq))
    free = np.nonzero(~solver.target_env(placements, scene.env_geoms()))[0]
    if free.size == 0:
        return valid, q
    sol = solver.solve(placements[free], q0, dtype="f64", eps=EPSILON, dt=DT_IK, max_iters=MAX_ITERS,
                       check_collision=True)
    ok = free[sol.converged.astype(bool)]
    q[free] = sol.q
    if ok.size:
        d = solver.distance(q[ok], placements[ok], scene.obstacle_pairs())
        valid[ok[d >= MIN_OBSTACLE_DISTANCE]] = True
    return valid, q


def sample_cube_placement(robot, cube, cubeplacementq0, cubeplacementqgoal, viz=None, batch=64):
    """path.py:27-62 (uniform sampler) -> (q, placement)."""
    (x0, x1), (y0, y1), (z0, z1) = _bounds(cubeplacementq0, cubeplacementqgoal)
    lo = np.array([x0, y0, z0])
    rng = np.array([x1 - x0, y1 - y0, z1 - z0])  # RandomState.uniform: low + (high - low) * u
    while True:
        state = np.random.get_state()
        u = np.random.random_sample((batch, 3))
        pts = lo + rng * u
        valid, q = _evaluate(robot, _rows(pts), robot.q0.copy())
        hit = np.nonzero(valid)[0]
        if hit.size == 0:
            continue  # the reference would have consumed the same 3 * batch draws
        i = int(hit[0])
        np.random.set_state(state)
        np.random.random_sample(3 * (i + 1))  # leave the stream where the sequential loop stops
        placement = SE3(np.eye(3), pts[i])
        setcubeplacement(robot, cube, placement)
        if viz is not None and hasattr(viz, "display"):
            viz.display(q[i])
        return q[i].copy(), placement


def sample_cube_placements(robot, cubeplacementq0, cubeplacementqgoal, n, rng=None, batch=1024):
    """n valid samples (q [n,nq], translations [n,3]) from a numpy Generator,
    evaluated `batch` candidates per round (no RandomState compatibility)."""
    rng = np.random.default_rng() if rng is None else rng
    (x0, x1), (y0, y1), (z0, z1) = _bounds(cubeplacementq0, cubeplacementqgoal)
    qs, ts = [], []
    while sum(len(t) for t in ts) < n:
        pts = np.stack([rng.uniform(x0, x1, batch), rng.uniform(y0, y1, batch), rng.uniform(z0, z1, batch)], 1)
        valid, q = _evaluate(robot, _rows(pts), robot.q0.copy())
        qs.append(q[valid])
        ts.append(pts[valid])
    return np.concatenate(qs)[:n], np.concatenate(ts)[:n]


def project_path(robot, cube, q_curr, cube_curr, cube_rand, step_size=0.025, viz=None):
    """path.py:125-163 -> (robot_path, cube_path), the valid prefix."""
    paths = project_paths(robot, [q_curr], [cube_curr], [cube_rand], step_size=step_size, cube=cube)
    if viz is not None and hasattr(viz, "display"):
        viz.display(paths[0][0][-1])
    return paths[0]


def project_paths(robot, q_currs, cube_currs, cube_rands, step_size=0.025, cube=None):
    """Many projections at once: chain c interpolates cube_currs[c] ->
    cube_rands[c] in int(|dt|/step_size)+1 steps (SE3.Interpolate), stops at
    the first cube/environment collision or failed IK, and warm-starts each
    solve from its previous q — the reference's loop per chain, with the
    active chains' step s solved in ONE batched launch.  Returns a list of
    (robot_path, cube_path)."""
    solver, scene = _solver_scene(robot)
    C = len(q_currs)
    env = scene.env_geoms()
    starts = [SE3(*as_rt(p)) for p in cube_currs]
    ends = [SE3(*as_rt(p)) for p in cube_rands]
    steps = [int(np.linalg.norm(a.translation - b.translation) / step_size) + 1 for a, b in zip(starts, ends)]
    robot_paths = [[np.array(q, dtype=np.float64)] for q in q_currs]
    cube_paths = [[p] for p in cube_currs]
    active = np.ones(C, dtype=bool)
    for s in range(1, max(steps) + 1):
        idx = [c for c in range(C) if active[c] and s <= steps[c]]
        if not idx:
            break
        pl = [interpolate(starts[c], ends[c], s / steps[c]) for c in idx]
        rows = np.stack([np.concatenate([p.rotation.reshape(9), p.translation]) for p in pl])
        col = solver.target_env(rows, env)
        go = [k for k in range(len(idx)) if not col[k]]
        for k in range(len(idx)):
            if col[k]:
                active[idx[k]] = False
        if not go:
            continue
        q0 = np.stack([robot_paths[idx[k]][-1] for k in go])
        sol = solver.solve(rows[go], q0, dtype="f64", eps=EPSILON, dt=DT_IK, max_iters=MAX_ITERS,
                           check_collision=True)
        for j, k in enumerate(go):
            c = idx[k]
            if not sol.converged[j]:
                active[c] = False
                continue
            robot_paths[c].append(sol.q[j].astype(np.float64))
            cube_paths[c].append(pl[k])
        if cube is not None and C == 1:
            setcubeplacement(robot, cube, pl[-1])  # the reference leaves the cube at the last attempt
    return [(robot_paths[c], cube_paths[c]) for c in range(C)]
