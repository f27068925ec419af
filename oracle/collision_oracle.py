"""CPU ORACLE (collision term) — test infrastructure only.

Restates the reference's collision check `tools.collision(robot, q)`
(tools.py:25-35: pin.updateGeometryPlacements + pin.computeCollisions over the
pairs built in setup_pinocchio.py:53-83) and the IK loop with that term
(inverse_geometry.py:70, :97-98).  hpp-fcl (the narrow phase the reference
calls) is not installed; its published semantics are restated: a pair
collides when the two convex shapes intersect (distance < 0).  Exact tests for
sphere/sphere, sphere/box and box/box (separating-axis theorem); GJK on
support functions for every pair involving a cylinder.  The cube mesh is its
convex hull (an 8-vertex box).

The scene (geometries, placements, active pairs) is parsed here independently
of the product's compiler (`ikgrasp/collision.py`) by `parse_scene`, frozen
into `tests/golden/collision_scene.json` by tests/golden/make_golden.py, and
the tests compare the two.

Parity: KAT-5 `collision(robot, robot.q0) == True` (lab_instructions.ipynb:252,
:262) and no collision at the KAT-1/KAT-2 solutions (their iteration counts
740/736 match the reference's charts only if the stop test passed there).
Beyond those, collision parity is UNPINNED (no hpp-fcl outputs exist in the
reference tree).
"""
from __future__ import annotations

import json
import math
import xml.etree.ElementTree as ET

import numpy as np

from . import ik_oracle as o

SPHERE, BOX, CYLINDER, MESHBOX = 0, 1, 2, 3


# ---------------------------------------------------------------- scene parsing
def _xyz_rpy(el):
    org = el.find("origin") if el is not None else None
    xyz = [float(v) for v in (org.get("xyz", "0 0 0") if org is not None else "0 0 0").split()]
    rpy = [float(v) for v in (org.get("rpy", "0 0 0") if org is not None else "0 0 0").split()]
    return o.urdf_rpy_to_matrix(*rpy), np.array(xyz)


def _collisions_dfs(path):
    """[(link, collision element)] in Pinocchio's depth-first link order."""
    root = ET.parse(path).getroot()
    kids = {}
    childs = set()
    for j in root.findall("joint"):
        kids.setdefault(j.find("parent").get("link"), []).append(j)
        childs.add(j.find("child").get("link"))
    links = {l.get("name"): l for l in root.findall("link")}
    start = [n for n in links if n not in childs][0]
    out, order = [], []

    def rec(name):
        order.append(name)
        for c in links[name].findall("collision"):
            out.append((name, c))
        for j in sorted(kids.get(name, []), key=lambda e: e.get("name")):
            rec(j.find("child").get("link"))

    rec(start)
    joints = {j.find("child").get("link"): j for j in root.findall("joint")}
    return out, joints


def _shape(c):
    g = list(c.find("geometry"))[0]
    if g.tag == "sphere":
        return SPHERE, [float(g.get("radius")), 0.0, 0.0]
    if g.tag == "box":
        return BOX, [0.5 * float(v) for v in g.get("size").split()]
    if g.tag == "cylinder":
        return CYLINDER, [float(g.get("radius")), 0.5 * float(g.get("length")), 0.0]
    return MESHBOX, [0.5 * float(v) for v in g.get("scale").split()]


def parse_scene(ref):
    """Geometries + active pairs of the reference scene (setuppinocchio)."""
    robot = f"{ref}/models/nextagea_description/urdf/NextageaOpen.urdf"
    names = [j[0] for j in o.JOINTS]
    cols, joints = _collisions_dfs(robot)
    geoms = []
    for k, (link, c) in enumerate(cols):
        # walk up fixed joints to the moving joint carrying this link
        R, t = np.eye(3), np.zeros(3)
        cur = link
        q = -1
        while cur in joints:
            j = joints[cur]
            if j.get("type") == "revolute":
                q = names.index(j.get("name"))
                break
            Rj, tj = _xyz_rpy(j)
            R, t = Rj @ R, tj + Rj @ t
            cur = j.find("parent").get("link")
        Rc, tc = _xyz_rpy(c)
        kind, dims = _shape(c)
        geoms.append({"kind": kind, "joint": q, "link": link, "R": R @ Rc, "t": t + R @ tc, "dims": dims,
                      "target": False})
    for g in geoms[:2]:  # translaterobot moves geometryObjects[0:2] only (setup_pinocchio.py:30-31)
        g["t"] = g["t"] + np.array([0.0, 0.0, o.ROBOT_Z])
    c, s = math.cos(-np.pi / 2), math.sin(-np.pi / 2)
    objs = [(f"{ref}/models/table/table_tallerscaled.urdf", np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]]),
             np.array([0.8, 0.0, 0.0]), False),
            (f"{ref}/models/cubes/obstacle.urdf", np.eye(3), np.array([0.43, -0.1, 0.94]), False),
            (f"{ref}/models/cubes/cube_small.urdf", np.eye(3), np.array([0.33, -0.3, 0.93]), True)]
    for path, Ro, to, tgt in objs:
        for link, cc in _collisions_dfs(path)[0]:
            Rc, tc = _xyz_rpy(cc)
            kind, dims = _shape(cc)
            geoms.append({"kind": kind, "joint": -1, "link": "base_link", "R": Ro @ Rc, "t": to + Ro @ tc,
                          "dims": dims, "target": tgt})
    srdf = ET.parse(f"{robot[:-len('NextageaOpen.urdf')]}NextageAOpen.srdf").getroot()
    off = {frozenset((d.get("link1"), d.get("link2"))) for d in srdf.findall("disable_collisions")}
    pairs = [(i, j) for i in range(len(geoms)) for j in range(i + 1, len(geoms))
             if geoms[i]["joint"] != geoms[j]["joint"]
             and frozenset((geoms[i]["link"], geoms[j]["link"])) not in off]
    pairs.append((len(geoms) - 2, len(geoms) - 1))  # CollisionPair(46, 47)
    return {"geoms": [{**g, "R": g["R"].tolist(), "t": g["t"].tolist()} for g in geoms], "pairs": pairs}


def load_scene(path):
    with open(path) as f:
        return prepare(json.load(f))


def prepare(d):
    """JSON-shaped scene (parse_scene / collision_scene.json) -> arrays, in place."""
    for g in d["geoms"]:
        g["R"] = np.array(g["R"])
        g["t"] = np.array(g["t"])
        g["dims"] = np.array(g["dims"], dtype=np.float64)
    d["pairs"] = [tuple(p) for p in d["pairs"]]
    return d


# ---------------------------------------------------------------- narrow phase
def support(g, R, t, d):
    k, dims = g["kind"], g["dims"]
    if k == SPHERE:
        n = np.linalg.norm(d)
        return t + (dims[0] * d / n if n > 0 else 0.0)
    dl = R.T @ d
    if k in (BOX, MESHBOX):
        return t + R @ (np.where(dl >= 0, 1.0, -1.0) * dims)
    rad = math.hypot(dl[0], dl[1])
    loc = np.array([dims[0] * dl[0] / rad if rad > 0 else 0.0, dims[0] * dl[1] / rad if rad > 0 else 0.0,
                    dims[1] if dl[2] >= 0 else -dims[1]])
    return t + R @ loc


def gjk_intersect(sa, sb, c0, max_iter=64):
    """Boolean GJK on the Minkowski difference A - B (support callables)."""
    def sup(d):
        return sa(d) - sb(-d)

    d = c0 if np.linalg.norm(c0) > 0 else np.array([1.0, 0.0, 0.0])
    simplex = [sup(d)]
    d = -simplex[0]
    for _ in range(max_iter):
        if np.dot(d, d) < 1e-30:
            return True
        a = sup(d)
        if np.dot(a, d) < 0:
            return False
        simplex.append(a)
        hit, simplex, d = _do_simplex(simplex)
        if hit:
            return True
    return True


def _do_simplex(s):
    a = s[-1]
    ao = -a
    if len(s) == 2:
        b = s[0]
        ab = b - a
        if np.dot(ab, ao) > 0:
            return False, [b, a], np.cross(np.cross(ab, ao), ab) if np.linalg.norm(np.cross(ab, ao)) > 1e-15 else \
                _perp(ab)
        return False, [a], ao
    if len(s) == 3:
        c, b = s[0], s[1]
        ab, ac = b - a, c - a
        abc = np.cross(ab, ac)
        if np.dot(np.cross(abc, ac), ao) > 0:
            if np.dot(ac, ao) > 0:
                return False, [c, a], np.cross(np.cross(ac, ao), ac)
            return _do_simplex([b, a])
        if np.dot(np.cross(ab, abc), ao) > 0:
            return _do_simplex([b, a])
        if np.dot(abc, ao) > 0:
            return False, [c, b, a], abc
        return False, [b, c, a], -abc
    d_, c, b = s[0], s[1], s[2]
    ab, ac, ad = b - a, c - a, d_ - a
    abc, acd, adb = np.cross(ab, ac), np.cross(ac, ad), np.cross(ad, ab)
    if np.dot(abc, ao) > 0:
        return _do_simplex([c, b, a])
    if np.dot(acd, ao) > 0:
        return _do_simplex([d_, c, a])
    if np.dot(adb, ao) > 0:
        return _do_simplex([b, d_, a])
    return True, s, ao


def _perp(v):
    t = np.array([1.0, 0, 0]) if abs(v[0]) < 0.9 else np.array([0, 1.0, 0])
    return np.cross(v, t)


def _box_box(R1, t1, h1, R2, t2, h2):
    """Separating-axis test for two oriented boxes (15 axes)."""
    axes = [R1[:, i] for i in range(3)] + [R2[:, i] for i in range(3)]
    axes += [np.cross(R1[:, i], R2[:, j]) for i in range(3) for j in range(3)]
    d = t2 - t1
    for ax in axes:
        n = np.linalg.norm(ax)
        if n < 1e-12:
            continue
        ax = ax / n
        r1 = sum(h1[i] * abs(np.dot(R1[:, i], ax)) for i in range(3))
        r2 = sum(h2[i] * abs(np.dot(R2[:, i], ax)) for i in range(3))
        if abs(np.dot(d, ax)) > r1 + r2:
            return False
    return True


def collide(ga, Ra, ta, gb, Rb, tb):
    ka, kb = ga["kind"], gb["kind"]
    if ka == SPHERE and kb == SPHERE:
        return np.linalg.norm(ta - tb) < ga["dims"][0] + gb["dims"][0]
    if ka == SPHERE and kb in (BOX, MESHBOX) or kb == SPHERE and ka in (BOX, MESHBOX):
        (gs, ts), (gx, Rx, tx) = ((ga, ta), (gb, Rb, tb)) if ka == SPHERE else ((gb, tb), (ga, Ra, ta))
        p = Rx.T @ (ts - tx)
        closest = np.clip(p, -gx["dims"], gx["dims"])
        return np.linalg.norm(p - closest) < gs["dims"][0]
    if ka in (BOX, MESHBOX) and kb in (BOX, MESHBOX):
        return _box_box(Ra, ta, ga["dims"], Rb, tb, gb["dims"])
    return gjk_intersect(lambda d: support(ga, Ra, ta, d), lambda d: support(gb, Rb, tb, d), ta - tb)


def geom_poses(scene, q, target_R, target_t):
    oMi = o.forward_kinematics(np.asarray(q, dtype=np.float64))
    poses = []
    for g in scene["geoms"]:
        if g["target"]:
            poses.append((np.asarray(target_R), np.asarray(target_t)))
        elif g["joint"] < 0:
            poses.append((g["R"], g["t"]))
        else:
            R, t = oMi[g["joint"]]
            poses.append((R @ g["R"], t + R @ g["t"]))
    return poses


def colliding_pairs(scene, q, target_R, target_t):
    poses = geom_poses(scene, q, target_R, target_t)
    gs = scene["geoms"]
    return [(i, j) for i, j in scene["pairs"]
            if collide(gs[i], poses[i][0], poses[i][1], gs[j], poses[j][0], poses[j][1])]


def collision(scene, q, target_R, target_t):
    """tools.collision (tools.py:25-35)."""
    poses = geom_poses(scene, q, target_R, target_t)
    gs = scene["geoms"]
    for i, j in scene["pairs"]:
        if collide(gs[i], poses[i][0], poses[i][1], gs[j], poses[j][0], poses[j][1]):
            return True
    return False


def computeqgrasppose(scene, q0, cube_R, cube_t, max_iters=o.MAX_ITERS, dt=o.DT, eps=o.EPSILON):
    """inverse_geometry.py:41-100 WITH the collision term (:70, :97-98)."""
    placements = o.joint_placements()
    oMcubeL, oMcubeR = o.hook_targets(cube_R, cube_t)
    q = np.array(q0, dtype=np.float64).copy()
    for it in range(max_iters):
        eL, eR = o.hand_errors(q, oMcubeL, oMcubeR, placements)
        nL, nR = np.linalg.norm(eL), np.linalg.norm(eR)
        if nL < eps and nR < eps and not collision(scene, q, cube_R, cube_t):
            return q, True, it, (nL, nR)
        JL = o.frame_jacobian_local(q, o.FRAME_LEFT, placements)
        JR = o.frame_jacobian_local(q, o.FRAME_RIGHT, placements)
        vq = np.linalg.pinv(np.vstack([JL, JR])) @ np.hstack([eL, eR])
        q = np.minimum(np.maximum(o.LOWER, q + vq * dt), o.UPPER)
    eL, eR = o.hand_errors(q, oMcubeL, oMcubeR, placements)
    return q, False, max_iters, (np.linalg.norm(eL), np.linalg.norm(eR))
