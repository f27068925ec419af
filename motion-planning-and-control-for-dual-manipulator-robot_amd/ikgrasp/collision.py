"""Collision scene compiler: URDF/SRDF -> flat tables for the collision
kernel (the collision term of `success`).

Restates what the reference builds (setup_pinocchio.py:53-83, tools.py:25-35):

* robot geometries: the URDF `<collision>` primitives of every link, in
  Pinocchio's depth-first link order (children by joint name), named
  `<link>_<k>`, placed in their parent joint frame (fixed joints folded);
* `translaterobot` (setup_pinocchio.py:28-32) premultiplies ROBOT_PLACEMENT
  into geometries 0 and 1 only (the base box and the first base sphere) — the
  other base spheres and the WAIST cylinder stay at URDF height (reference
  quirk, reproduced);
* `loadobject` appends the table, obstacle and cube geometries placed by
  TABLE/OBSTACLE/CUBE_PLACEMENT (config.py:34-36); the cube's placement is
  overwritten per solve by `setcubeplacement` (tools.py:62-68) — here it is the
  solve's target;
* pairs (`finalisecollisionsetup`, setup_pinocchio.py:53-60):
  `addAllCollisionPairs` = every pair with different parent joints, minus the
  SRDF `<disable_collisions>` entries matched on body frames, plus (46, 47)
  (obstacle, cube).  The scene objects keep the frame index 1 of their own
  models, which in the robot model is `base_link`; no SRDF entry names it, so
  no scene pair is removed.

Geometry kinds (hpp-fcl shapes): 0 sphere (radius), 1 box (half extents),
2 cylinder (radius, half length along local z), 3 triangle-mesh cube treated
as its convex hull box (cube.obj scaled by 0.1: an 8-vertex box).
"""
from __future__ import annotations

import json
import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

from .model import DATA_DIR, _compose, _floats, _origin, rpy_to_matrix

SPHERE, BOX, CYLINDER, MESHBOX = 0, 1, 2, 3


@dataclass
class Geom:
    name: str
    kind: int
    joint: int            # q index of the parent joint, -1 = universe
    frame: str            # body (link) name used for SRDF matching
    R: np.ndarray         # placement in the parent joint frame (world if joint == -1)
    t: np.ndarray
    dims: np.ndarray      # [3]
    target: bool = False  # placement = the solve's cube target (setcubeplacement)


@dataclass
class CollisionScene:
    geoms: list = field(default_factory=list)
    pairs: np.ndarray = None  # [N, 2] int

    def to_json(self) -> str:
        return json.dumps({
            "geoms": [{"name": g.name, "kind": g.kind, "joint": g.joint, "frame": g.frame,
                       "R": g.R.tolist(), "t": g.t.tolist(), "dims": g.dims.tolist(), "target": g.target}
                      for g in self.geoms],
            "pairs": self.pairs.tolist(),
        }, indent=1)

    def geom_id(self, name: str) -> int:
        """robot.collision_model.getGeometryId(name)"""
        for i, g in enumerate(self.geoms):
            if g.name == name:
                return i
        raise KeyError(name)

    def obstacle_pairs(self, obstacle="obstaclebase_0", table="baseLink_0") -> np.ndarray:
        """tools.py:39-41: active pairs whose second geometry is the obstacle or the table."""
        ids = {self.geom_id(obstacle), self.geom_id(table)}
        return np.array([k for k, (_, j) in enumerate(self.pairs) if int(j) in ids], dtype=np.int32)

    def env_geoms(self, table="baseLink_0", obstacle="obstaclebase_0") -> np.ndarray:
        """The cube's collision model partners (setup_pinocchio.py:62-70): table, obstacle."""
        return np.array([self.geom_id(table), self.geom_id(obstacle)], dtype=np.int32)

    @staticmethod
    def from_json(text: str) -> "CollisionScene":
        d = json.loads(text)
        geoms = [Geom(g["name"], g["kind"], g["joint"], g["frame"], np.array(g["R"]), np.array(g["t"]),
                      np.array(g["dims"]), g["target"]) for g in d["geoms"]]
        return CollisionScene(geoms, np.array(d["pairs"], dtype=np.int32).reshape(-1, 2))


def _shape(geom_el, scale_mesh=None):
    g = list(geom_el)[0]
    if g.tag == "sphere":
        return SPHERE, np.array([float(g.get("radius")), 0.0, 0.0])
    if g.tag == "box":
        return BOX, np.array(_floats(g.get("size"), 3, None)) / 2.0
    if g.tag == "cylinder":
        return CYLINDER, np.array([float(g.get("radius")), float(g.get("length")) / 2.0, 0.0])
    if g.tag == "mesh":
        s = np.array(_floats(g.get("scale"), 3, (1.0, 1.0, 1.0)))
        # cube.obj: vertices at +-0.5 (a unit cube) -> half extents 0.5 * scale
        return MESHBOX, 0.5 * s
    raise ValueError(f"unsupported collision geometry {g.tag}")


def _link_geoms(root, joint_index_of_link):
    """Geometries of a URDF in Pinocchio's DFS link order, with placement in
    the parent joint frame.  `joint_index_of_link(link) -> (q index, link-in-joint)`."""
    links = {l.get("name"): l for l in root.findall("link")}
    children = {}
    child_links = set()
    for j in root.findall("joint"):
        children.setdefault(j.find("parent").get("link"), []).append(j)
        child_links.add(j.find("child").get("link"))
    root_link = sorted(set(links) - child_links)[0]
    out = []

    def visit(link):
        joint, link_in_joint = joint_index_of_link(link)
        for k, c in enumerate(links[link].findall("collision")):
            kind, dims = _shape(c.find("geometry"))
            R, t = _compose(link_in_joint, _origin(c))
            out.append(Geom(f"{link}_{k}", kind, joint, link, R, t, dims))
        for j in sorted(children.get(link, []), key=lambda e: e.get("name")):
            visit(j.find("child").get("link"))

    visit(root_link)
    return out


def _robot_link_frames(root, joint_names, axis_frames=None):
    """link -> (q index of its parent joint or -1, link placement in that joint frame).
    axis_frames: the model's joint-frame changes Q (DualArmModel.axis_frames(),
    non-canonical axes): a revolute joint's child link sits at Q^T in its frame."""
    joints = {j.get("name"): j for j in root.findall("joint")}
    parent_joint = {}
    for j in joints.values():
        parent_joint[j.find("child").get("link")] = j
    cache = {}

    def resolve(link):
        if link in cache:
            return cache[link]
        j = parent_joint.get(link)
        if j is None:
            res = (-1, (np.eye(3), np.zeros(3)))
        elif j.get("type") == "revolute":
            q = joint_names.index(j.get("name"))
            res = (q, (np.eye(3) if axis_frames is None else np.asarray(axis_frames[q]).T, np.zeros(3)))
        else:  # fixed: fold the origin into the parent's frame
            pj, pM = resolve(j.find("parent").get("link"))
            res = (pj, _compose(pM, _origin(j)))
        cache[link] = res
        return res

    return resolve


def build_scene(robot_urdf, srdf, table_urdf, obstacle_urdf, cube_urdf, joint_names, robot_placement,
                table_placement, obstacle_placement, cube_placement, axis_frames=None) -> CollisionScene:
    """Placements are (R, t) tuples (config.py:33-37); axis_frames = the
    robot model's DualArmModel.axis_frames() (identity for the Nextage)."""
    rroot = ET.parse(robot_urdf).getroot()
    geoms = _link_geoms(rroot, _robot_link_frames(rroot, joint_names, axis_frames))
    # translaterobot: only geometryObjects[0:2] are moved (setup_pinocchio.py:30-31)
    for g in geoms[:2]:
        g.R, g.t = _compose(robot_placement, (g.R, g.t))
    for path, M, is_cube in ((table_urdf, table_placement, False), (obstacle_urdf, obstacle_placement, False),
                             (cube_urdf, cube_placement, True)):
        oroot = ET.parse(path).getroot()
        for g in _link_geoms(oroot, lambda link: (-1, (np.eye(3), np.zeros(3)))):
            g.R, g.t = _compose(M, (g.R, g.t))  # setup_pinocchio.translate
            g.frame = "base_link"  # frame index 1 of the object's own model == robot frame 1
            g.target = is_cube
            geoms.append(g)
    n = len(geoms)
    disabled = set()
    for dc in ET.parse(srdf).getroot().findall("disable_collisions"):
        disabled.add(frozenset((dc.get("link1"), dc.get("link2"))))
    pairs = []
    for i in range(n):
        for j in range(i + 1, n):
            if geoms[i].joint == geoms[j].joint:
                continue
            if frozenset((geoms[i].frame, geoms[j].frame)) in disabled and geoms[i].frame != geoms[j].frame:
                continue
            pairs.append((i, j))
    obstacle = next(k for k, g in enumerate(geoms) if g.name.startswith("obstaclebase"))
    cube = next(k for k, g in enumerate(geoms) if g.target)
    if (obstacle, cube) not in pairs:
        pairs.append((obstacle, cube))  # setup_pinocchio.py:58 CollisionPair(46, 47)
    return CollisionScene(geoms, np.array(pairs, dtype=np.int32))


NEXTAGE_COLLISION_JSON = os.path.join(DATA_DIR, "nextage_collision.json")


def load_nextage_scene() -> CollisionScene:
    with open(NEXTAGE_COLLISION_JSON) as f:
        return CollisionScene.from_json(f.read())
