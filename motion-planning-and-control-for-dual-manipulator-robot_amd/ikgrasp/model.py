"""Kinematic model compiler: URDF -> flat dual-arm tables for the HIP kernel.

Restates what Pinocchio's URDF parser builds for the reference
(`setup_pinocchio.py:73-83` -> `RobotWrapper.BuildFromURDF`, then
`translaterobot` at :28-32):

* revolute joints become Pinocchio joints in depth-first order from the root
  link, children visited in urdfdom's `std::map` order (sorted by joint name);
  the order is pinned by `lab_instructions.ipynb:210-226`;
* fixed joints are merged: their origin is folded into the placement of the
  next movable joint, and they also define frames (`LARM_EFF`, the cube hooks);
* `<origin rpy>` is converted through urdfdom's quaternion and Eigen's
  `Quaterniond::matrix()` (the path `pinocchio::urdf::convertFromUrdf` takes);
* the robot base placement (`config.py:33` ROBOT_PLACEMENT) is premultiplied
  into the placement of joint 1 (`setup_pinocchio.py:32`).

The kernel's structural contract (checked in `DualArmModel.validate`): one
shared root joint (the chest) followed by two 6-joint arm chains ending in
the left/right effector frames; all other joints are passive (never moved by
the IK, only clamped, as the reference's zero Jacobian columns imply).

Joint axes.  +X/+Y/+Z become Pinocchio's RX/RY/RZ joints;
any other direction e (a negative or tilted axis: Pinocchio's
RevoluteUnaligned, rotation exp(q [e]x)) is compiled onto the canonical axis c
nearest to it by re-expressing the joint's frame: with Q c = e,
Rot(e, q) = Q Rot(c, q) Q^T, so the joint gets placement Q_parent^T P Q and
axis c, and everything attached to it (child joint placements, frames,
collision geometries) is premultiplied by Q^T.  World placements of every
frame and geometry, the joint origins and world axes -- hence FK, every frame
Jacobian and the IK iterates -- are unchanged, while the kernels keep their
compile-time canonical-axis rotations.
"""
from __future__ import annotations

import json
import math
import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

ARM_DOF = 6


def rpy_to_matrix(r: float, p: float, y: float) -> np.ndarray:
    """urdfdom `Rotation::setFromRPY` + normalize, then Eigen quaternion -> matrix."""
    hr, hp, hy = r / 2.0, p / 2.0, y / 2.0
    sr, cr = math.sin(hr), math.cos(hr)
    sp, cp = math.sin(hp), math.cos(hp)
    sy, cy = math.sin(hy), math.cos(hy)
    x = sr * cp * cy - cr * sp * sy
    yq = cr * sp * cy + sr * cp * sy
    z = cr * cp * sy - sr * sp * cy
    w = cr * cp * cy + sr * sp * sy
    n = math.sqrt(x * x + yq * yq + z * z + w * w)
    x, yq, z, w = x / n, yq / n, z / n, w / n
    tx, ty, tz = 2.0 * x, 2.0 * yq, 2.0 * z
    return np.array([
        [1.0 - (ty * yq + tz * z), ty * x - tz * w, tz * x + ty * w],
        [ty * x + tz * w, 1.0 - (tx * x + tz * z), tz * yq - tx * w],
        [tz * x - ty * w, tz * yq + tx * w, 1.0 - (tx * x + ty * yq)],
    ])


def _floats(s, n, default):
    if s is None:
        return list(default)
    v = [float(t) for t in s.split()]
    if len(v) != n:
        raise ValueError(f"expected {n} numbers, got {s!r}")
    return v


def _origin(el):
    o = el.find("origin")
    xyz = _floats(o.get("xyz") if o is not None else None, 3, (0.0, 0.0, 0.0))
    rpy = _floats(o.get("rpy") if o is not None else None, 3, (0.0, 0.0, 0.0))
    return rpy_to_matrix(*rpy), np.array(xyz, dtype=np.float64)


def _compose(A, B):
    return (A[0] @ B[0], A[1] + A[0] @ B[1])


@dataclass
class Joint:
    name: str
    parent: int          # parent joint index (-1 = universe), in q order
    R: np.ndarray        # placement in the parent joint frame
    t: np.ndarray
    axis: int            # 0/1/2 = X/Y/Z: the kernel's canonical axis
    lower: float
    upper: float
    axis_dir: np.ndarray = None  # the URDF axis, normalised
    Q: np.ndarray = None         # joint-frame change with Q e_axis = axis_dir (I when aligned)


def _unit(k: int) -> np.ndarray:
    e = np.zeros(3)
    e[k] = 1.0
    return e


def axis_frame(e: np.ndarray):
    """(canonical axis code c, rotation Q with Q e_c = e) for a unit axis e:
    Q = I for +X/+Y/+Z; a half turn about the next canonical axis for -X/-Y/-Z
    (exact); otherwise the minimal rotation from e_c (c = largest |e_i|) to e."""
    c = int(np.argmax(np.abs(e)))
    u = _unit(c)
    if np.array_equal(e, u):
        return c, np.eye(3)
    if np.array_equal(e, -u):
        Q = -np.eye(3)
        k = (c + 1) % 3
        Q[k, k] = 1.0  # rotation by pi about axis k: diag(+1 on k, -1 elsewhere)
        return c, Q
    k = np.cross(u, e)
    s2 = float(k @ k)
    K = np.array([[0.0, -k[2], k[1]], [k[2], 0.0, -k[0]], [-k[1], k[0], 0.0]])
    return c, np.eye(3) + K + K @ K * ((1.0 - float(u @ e)) / s2)


@dataclass
class Frame:
    name: str
    parent: int          # parent joint index (-1 = universe)
    R: np.ndarray
    t: np.ndarray


@dataclass
class KinematicTree:
    joints: list = field(default_factory=list)
    frames: dict = field(default_factory=dict)

    @property
    def nq(self) -> int:
        return len(self.joints)

    def joint_names(self):
        return [j.name for j in self.joints]


def parse_urdf(path_or_xml: str, base_placement=None) -> KinematicTree:
    """Parse a URDF (path or XML text) into Pinocchio-ordered joints and frames."""
    if os.path.exists(path_or_xml):
        root = ET.parse(path_or_xml).getroot()
    else:
        root = ET.fromstring(path_or_xml)
    links = {l.get("name") for l in root.findall("link")}
    joints = {}
    children = {}
    child_links = set()
    for j in root.findall("joint"):
        name = j.get("name")
        parent = j.find("parent").get("link")
        child = j.find("child").get("link")
        joints[name] = j
        children.setdefault(parent, []).append(name)
        child_links.add(child)
    roots = sorted(links - child_links)
    if len(roots) != 1:
        raise ValueError(f"URDF must have exactly one root link, found {roots}")
    tree = KinematicTree()
    identity = (np.eye(3), np.zeros(3))
    # the root link's body frame sits at the universe origin
    tree.frames[roots[0]] = Frame(roots[0], -1, np.eye(3), np.zeros(3))

    def visit(link, parent_joint, link_in_parent):
        # urdfdom stores joints in a std::map -> child joints sorted by name
        for jname in sorted(children.get(link, [])):
            j = joints[jname]
            jtype = j.get("type")
            child = j.find("child").get("link")
            origin = _compose(link_in_parent, _origin(j))
            if jtype == "fixed":
                tree.frames[jname] = Frame(jname, parent_joint, origin[0], origin[1])
                tree.frames[child] = Frame(child, parent_joint, origin[0], origin[1])
                visit(child, parent_joint, origin)
            elif jtype == "revolute":
                ax = np.array(_floats(j.find("axis").get("xyz") if j.find("axis") is not None else None,
                                      3, (1.0, 0.0, 0.0)))
                nrm = float(np.linalg.norm(ax))
                if not nrm > 0.0:
                    raise ValueError(f"joint {jname}: zero axis")
                e = ax / nrm
                code, Q = axis_frame(e)
                lim = j.find("limit")
                lower = float(lim.get("lower", "0")) if lim is not None else 0.0
                upper = float(lim.get("upper", "0")) if lim is not None else 0.0
                R, t = origin
                if parent_joint < 0 and base_placement is not None:
                    R, t = _compose(base_placement, (R, t))
                tree.joints.append(Joint(jname, parent_joint, R, t, code, lower, upper, e, Q))
                idx = len(tree.joints) - 1
                tree.frames[jname] = Frame(jname, idx, np.eye(3), np.zeros(3))
                tree.frames[child] = Frame(child, idx, np.eye(3), np.zeros(3))
                visit(child, idx, identity)
            else:
                raise ValueError(f"joint {jname}: type {jtype!r} unsupported by the IK kernel")

    visit(roots[0], -1, identity)
    # re-express every joint frame so that its axis is canonical (module doc):
    # placement P -> Q_parent^T P Q, anything attached to joint j -> Q_j^T (.)
    Qs = [jt.Q for jt in tree.joints]
    for jt in tree.joints:
        Qp = Qs[jt.parent] if jt.parent >= 0 else np.eye(3)
        jt.R, jt.t = Qp.T @ jt.R @ jt.Q, Qp.T @ jt.t
    for f in tree.frames.values():
        if f.parent >= 0:
            f.R, f.t = Qs[f.parent].T @ f.R, Qs[f.parent].T @ f.t
    return tree


@dataclass
class DualArmModel:
    """Flat tables consumed by `ikg_model_create` (include/ikgrasp.h)."""
    joint_names: list
    parents: list
    R: np.ndarray            # [nq,3,3] joint placements
    t: np.ndarray            # [nq,3]
    axis: np.ndarray         # [nq] int
    lower: np.ndarray        # [nq]
    upper: np.ndarray        # [nq]
    root_q: int              # shared (chest) joint
    arm_q: np.ndarray        # [2,6] q indices, proximal -> distal
    hand_R: np.ndarray       # [2,3,3] effector frame in the last arm joint frame
    hand_t: np.ndarray       # [2,3]
    hook_R: np.ndarray       # [2,3,3] grasp hooks in the cube frame
    hook_t: np.ndarray       # [2,3]
    hand_names: tuple = ("LARM_EFF", "RARM_EFF")
    hook_names: tuple = ("LARM_HOOK", "RARM_HOOK")
    Q: np.ndarray = None     # [nq,3,3] joint-frame changes of non-canonical axes (parse_urdf); I if None

    def axis_frames(self) -> np.ndarray:
        return np.stack([np.eye(3)] * self.nq) if self.Q is None else self.Q

    @property
    def nq(self) -> int:
        return len(self.joint_names)

    @property
    def passive_q(self):
        active = {self.root_q, *self.arm_q.reshape(-1).tolist()}
        return [i for i in range(self.nq) if i not in active]

    def validate(self):
        for a in range(2):
            chain = [self.root_q] + self.arm_q[a].tolist()
            for k in range(1, len(chain)):
                if self.parents[chain[k]] != chain[k - 1]:
                    raise ValueError("arm chains must hang off the shared root joint as serial chains")
        if self.parents[self.root_q] != -1:
            raise ValueError("the shared joint must be the first joint below the universe")
        return self

    @staticmethod
    def from_trees(robot: KinematicTree, cube: KinematicTree, hands=("LARM_EFF", "RARM_EFF"),
                   hooks=("LARM_HOOK", "RARM_HOOK")) -> "DualArmModel":
        parents = [j.parent for j in robot.joints]
        chains = []
        for h in hands:
            f = robot.frames[h]
            chain = []
            i = f.parent
            while i >= 0:
                chain.append(i)
                i = parents[i]
            chains.append(chain[::-1])
        common = 0
        while common < min(map(len, chains)) and chains[0][common] == chains[1][common]:
            common += 1
        if common != 1:
            raise ValueError(f"kernel needs exactly one shared joint before the arms, found {common}")
        arms = [c[1:] for c in chains]
        if any(len(a) != ARM_DOF for a in arms):
            raise ValueError(f"kernel needs {ARM_DOF}-joint arms, got {[len(a) for a in arms]}")
        if any(robot.joints[arms[0][k]].axis != robot.joints[arms[1][k]].axis for k in range(ARM_DOF)):
            raise ValueError("left/right arm axis patterns must match (lane-uniform joint types)")
        hand_R = np.stack([robot.frames[h].R for h in hands])
        hand_t = np.stack([robot.frames[h].t for h in hands])
        # hooks: cube has no joints; frames hang off the universe
        hook_R = np.stack([cube.frames[h].R for h in hooks])
        hook_t = np.stack([cube.frames[h].t for h in hooks])
        return DualArmModel(
            joint_names=robot.joint_names(), parents=parents,
            R=np.stack([j.R for j in robot.joints]), t=np.stack([j.t for j in robot.joints]),
            axis=np.array([j.axis for j in robot.joints], dtype=np.int32),
            lower=np.array([j.lower for j in robot.joints]), upper=np.array([j.upper for j in robot.joints]),
            root_q=chains[0][0], arm_q=np.array(arms, dtype=np.int32),
            hand_R=hand_R, hand_t=hand_t, hook_R=hook_R, hook_t=hook_t,
            hand_names=tuple(hands), hook_names=tuple(hooks),
            Q=np.stack([j.Q for j in robot.joints])).validate()

    @staticmethod
    def from_urdf(robot_urdf: str, cube_urdf: str, base_placement=None, **kw) -> "DualArmModel":
        return DualArmModel.from_trees(parse_urdf(robot_urdf, base_placement), parse_urdf(cube_urdf), **kw)

    # ---- serialisation (the GPU box has no reference tree: ship compiled tables)
    def to_json(self) -> str:
        d = {
            "joint_names": self.joint_names, "parents": self.parents,
            "R": self.R.tolist(), "t": self.t.tolist(), "axis": self.axis.tolist(),
            "lower": self.lower.tolist(), "upper": self.upper.tolist(),
            "root_q": int(self.root_q), "arm_q": self.arm_q.tolist(),
            "hand_R": self.hand_R.tolist(), "hand_t": self.hand_t.tolist(),
            "hook_R": self.hook_R.tolist(), "hook_t": self.hook_t.tolist(),
            "hand_names": list(self.hand_names), "hook_names": list(self.hook_names),
            "Q": self.axis_frames().tolist(),
        }
        return json.dumps(d, indent=1)

    @staticmethod
    def from_json(text: str) -> "DualArmModel":
        d = json.loads(text)
        return DualArmModel(
            joint_names=d["joint_names"], parents=d["parents"],
            R=np.array(d["R"]), t=np.array(d["t"]), axis=np.array(d["axis"], dtype=np.int32),
            lower=np.array(d["lower"]), upper=np.array(d["upper"]),
            root_q=d["root_q"], arm_q=np.array(d["arm_q"], dtype=np.int32),
            hand_R=np.array(d["hand_R"]), hand_t=np.array(d["hand_t"]),
            hook_R=np.array(d["hook_R"]), hook_t=np.array(d["hook_t"]),
            hand_names=tuple(d["hand_names"]), hook_names=tuple(d["hook_names"]),
            Q=np.array(d["Q"]) if "Q" in d else None).validate()


DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
NEXTAGE_JSON = os.path.join(DATA_DIR, "nextage_dualarm.json")


def load_nextage() -> DualArmModel:
    """The Nextage + small-cube model of the reference scene (compiled by
    `tools/compile_model.py` from the reference URDFs)."""
    with open(NEXTAGE_JSON) as f:
        return DualArmModel.from_json(f.read())
