"""CPU ORACLE — test infrastructure only, never the product path.

Restatement of the planner-side queries of SURVEY §8f-2 that call the IK:
  * `distance_to_obstacle`   tools.py:37-51 (hpp-fcl computeDistance over the
                             active pairs whose second geometry is the table
                             or the obstacle);
  * `target_env`             path.py:51-52 / :136-138 (pin.computeCollisions on
                             the cube's own collision model,
                             setup_pinocchio.py:62-70: cube vs table, cube vs
                             obstacle);
  * `se3_interpolate`        pin.SE3.Interpolate (path.py:141):
                             A * exp6(alpha * log6(A^-1 B));
  * `sample_cube_placement`  path.py:27-62 (uniform sampler);
  * `project_path`           path.py:125-163.
Only `tests/` (and tests/golden/make_golden.py) may import this module.

The pair distance is computed WITHOUT GJK, so it checks the product's GJK
independently: exactly for sphere/sphere and sphere/box, as a bound-
constrained linear least-squares problem for box/box (scipy lsq_linear,
BVLS), and as a convex program (SLSQP) when a cylinder is involved.
hpp-fcl itself is absent from this image, so distance parity against hpp-fcl
is unpinned; hpp-fcl's published distance is the Euclidean distance between
the two separated convex shapes, which is what is restated here.
"""
from __future__ import annotations

import math

import numpy as np
from scipy.optimize import lsq_linear, minimize

from oracle import collision_oracle as co
from oracle import ik_oracle as o

SPHERE, BOX, CYLINDER, MESHBOX = co.SPHERE, co.BOX, co.CYLINDER, co.MESHBOX


# ---------------------------------------------------------------- pair distance
def _box_box_distance(Ra, ta, ha, Rb, tb, hb):
    # min |ta + Ra u - tb - Rb v|, |u_i| <= ha_i, |v_i| <= hb_i  (BVLS)
    A = np.hstack([Ra, -Rb])
    b = tb - ta
    lo = np.concatenate([-ha, -hb])
    res = lsq_linear(A, b, bounds=(lo, -lo), method="bvls", tol=1e-15, lsmr_tol=None)
    r = A @ res.x - b
    return float(np.linalg.norm(r))


def _convex_point(g, R, t):
    """(n_vars, point(x), constraints) of a shape in local parameters."""
    k, dims = g["kind"], g["dims"]
    if k == SPHERE:  # the centre (radius subtracted by the caller)
        return 0, (lambda x: t), [], []
    if k in (BOX, MESHBOX):
        return 3, (lambda x: t + R @ x), [(-dims[i], dims[i]) for i in range(3)], []
    r, h = dims[0], dims[1]
    cons = [{"type": "ineq", "fun": lambda x, r=r: r * r - x[0] * x[0] - x[1] * x[1],
             "jac": lambda x: np.array([-2 * x[0], -2 * x[1], 0.0])}]
    return 3, (lambda x: t + R @ x), [(-r, r), (-r, r), (-h, h)], cons


def _slsqp_distance(ga, Ra, ta, gb, Rb, tb):
    na, pa, ba, ca = _convex_point(ga, Ra, ta)
    nb, pb, bb, cb = _convex_point(gb, Rb, tb)

    def split(x):
        return x[:na], x[na:]

    def f(x):
        xa, xb = split(x)
        d = pa(xa) - pb(xb)
        return float(d @ d)

    def jac(x):
        xa, xb = split(x)
        d = 2.0 * (pa(xa) - pb(xb))
        ja = Ra.T @ d if na else np.zeros(0)
        jb = -(Rb.T @ d) if nb else np.zeros(0)
        return np.concatenate([ja, jb])

    cons = []
    for c in ca:
        cons.append({"type": "ineq", "fun": (lambda x, c=c: c["fun"](x[:na])),
                     "jac": (lambda x, c=c: np.concatenate([c["jac"](x[:na]), np.zeros(nb)]))})
    for c in cb:
        cons.append({"type": "ineq", "fun": (lambda x, c=c: c["fun"](x[na:])),
                     "jac": (lambda x, c=c: np.concatenate([np.zeros(na), c["jac"](x[na:])]))})
    x0 = np.zeros(na + nb)
    best = None
    for _ in range(2):  # restart from the first solution (SLSQP polish)
        res = minimize(f, x0, jac=jac, bounds=ba + bb, constraints=cons, method="SLSQP",
                       options={"ftol": 1e-20, "maxiter": 500})
        x0 = res.x
        best = res.fun if best is None else min(best, res.fun)
    return math.sqrt(max(best, 0.0))


def pair_distance(ga, Ra, ta, gb, Rb, tb):
    """min_distance of one pair (<= 0 when the shapes intersect)."""
    ka, kb = ga["kind"], gb["kind"]
    ra = ga["dims"][0] if ka == SPHERE else 0.0
    rb = gb["dims"][0] if kb == SPHERE else 0.0
    if ka == SPHERE and kb == SPHERE:
        return float(np.linalg.norm(ta - tb)) - ra - rb
    if (ka == SPHERE and kb in (BOX, MESHBOX)) or (kb == SPHERE and ka in (BOX, MESHBOX)):
        (gs, ts), (gx, Rx, tx) = ((ga, ta), (gb, Rb, tb)) if ka == SPHERE else ((gb, tb), (ga, Ra, ta))
        p = Rx.T @ (ts - tx)
        return float(np.linalg.norm(p - np.clip(p, -gx["dims"], gx["dims"]))) - gs["dims"][0]
    if ka in (BOX, MESHBOX) and kb in (BOX, MESHBOX):
        return _box_box_distance(Ra, ta, ga["dims"], Rb, tb, gb["dims"])
    return _slsqp_distance(ga, Ra, ta, gb, Rb, tb) - ra - rb


# ---------------------------------------------------------------- scene queries
def env_ids(scene):
    """(table, obstacle): the scene's objects added after the robot, in
    setuppinocchio's order (table 'baseLink_0', obstacle 'obstaclebase_0',
    setup_pinocchio.py:75-77); the oracle's scene reader keeps no names."""
    env = [i for i, g in enumerate(scene["geoms"])
           if g["joint"] < 0 and g["link"] == "base_link" and not g["target"]]
    assert len(env) == 2, env
    return env[0], env[1]


def obstacle_pairs(scene):
    """tools.py:39-41: pairs whose second geometry is the obstacle or the table."""
    ids = set(env_ids(scene))
    return [k for k, (_, j) in enumerate(scene["pairs"]) if j in ids]


def pair_distances(scene, q, target_R, target_t, pair_idx):
    poses = co.geom_poses(scene, q, target_R, target_t)
    gs = scene["geoms"]
    out = []
    for k in pair_idx:
        i, j = scene["pairs"][k]
        out.append(pair_distance(gs[i], poses[i][0], poses[i][1], gs[j], poses[j][0], poses[j][1]))
    return np.array(out)


def distance_to_obstacle(scene, q, target_R, target_t):
    """tools.distanceToObstacle (tools.py:37-51)."""
    return float(pair_distances(scene, q, target_R, target_t, obstacle_pairs(scene)).min())


def target_env(scene, target_R, target_t):
    """path.py:51-52: cube (at the placement) vs table, cube vs obstacle."""
    gs = scene["geoms"]
    cube = next(i for i, g in enumerate(gs) if g["target"])
    for j in env_ids(scene):
        if co.collide(gs[cube], np.asarray(target_R), np.asarray(target_t), gs[j], gs[j]["R"], gs[j]["t"]):
            return True
    return False


# ---------------------------------------------------------------- SE3.Interpolate
def exp6(v):
    """pin.exp6 of [v; w] (Pinocchio spatial/explog.hpp)."""
    lin, w = np.asarray(v[:3], dtype=np.float64), np.asarray(v[3:], dtype=np.float64)
    t2 = float(w @ w)
    t = math.sqrt(t2)
    prec3 = np.finfo(np.float64).eps ** 0.25
    if t < prec3:
        a = 1.0 - t2 / 6.0
        b = 0.5 - t2 / 24.0
        c = 1.0 / 6.0 - t2 / 120.0
    else:
        st, ct = math.sin(t), math.cos(t)
        a = st / t
        b = (1.0 - ct) / t2
        c = (t - st) / (t2 * t)
    W = np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])
    R = np.eye(3) + a * W + b * (W @ W)
    V = np.eye(3) + b * W + c * (W @ W)
    return R, V @ lin


def se3_interpolate(A, B, alpha):
    """pin.SE3.Interpolate(A, B, alpha) = A * exp6(alpha * log6(A^-1 B))."""
    dv = o.log6(o.se3_mul(o.se3_inv(A), B))
    return o.se3_mul(A, exp6(alpha * dv))


# ---------------------------------------------------------------- sampler / projection
def sample_cube_placement(scene, rs, cube_q0_t, cube_goal_t, min_obstacle_distance=0.04, max_attempts=1000):
    """path.py:27-62 (uniform sampler) with the numpy RandomState `rs` standing
    for the reference's global np.random.  Returns (q, t, attempts)."""
    x_min, x_max = min(cube_q0_t[0], cube_goal_t[0]), max(cube_q0_t[0], cube_goal_t[0])
    y_min, y_max = min(cube_q0_t[1], cube_goal_t[1]), max(cube_q0_t[1], cube_goal_t[1])
    z_min, z_max = 1.05, 1.4
    I = np.eye(3)
    for attempt in range(1, max_attempts + 1):
        x = rs.uniform(x_min, x_max)
        y = rs.uniform(y_min, y_max)
        z = rs.uniform(z_min, z_max)
        t = np.array([x, y, z])
        if target_env(scene, I, t):
            continue
        q, ok, _, _ = co.computeqgrasppose(scene, np.zeros(o.NQ), I, t)
        if ok and distance_to_obstacle(scene, q, I, t) >= min_obstacle_distance:
            return q, t, attempt
    raise RuntimeError("no valid placement")


def project_path(scene, q_curr, cube_curr, cube_rand, step_size=0.025):
    """path.py:125-163: (robot_path, cube_path) up to the first failure."""
    distance = np.linalg.norm(cube_curr[1] - cube_rand[1])
    num_steps = int(distance / step_size) + 1
    robot_path, cube_path = [np.asarray(q_curr, dtype=np.float64)], [cube_curr]
    for step in range(1, num_steps + 1):
        P = se3_interpolate(cube_curr, cube_rand, step / num_steps)
        if target_env(scene, P[0], P[1]):
            return robot_path, cube_path
        q, ok, _, _ = co.computeqgrasppose(scene, robot_path[-1].copy(), P[0], P[1])
        if not ok:
            return robot_path, cube_path
        robot_path.append(q)
        cube_path.append(P)
    return robot_path, cube_path
