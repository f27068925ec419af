"""Tables from a Pinocchio `RobotWrapper` (or any object with its attribute
surface), so the drop-in `computeqgrasppose` accepts the reference's own
`robot` and `cube` (SURVEY §8b "Duck typing"; the objects built by
/root/reference/setup_pinocchio.py:73-83).

Nothing here imports Pinocchio.  What is read:

* `robot.model`: `njoints`, `names`, `parents`, `jointPlacements[j]`
  (`.rotation`, `.translation`; joint 1's already carries ROBOT_PLACEMENT after
  `translaterobot`, setup_pinocchio.py:32), `joints[j].shortname()` (RX / RY /
  RZ, or RevoluteUnaligned with `.axis`), `joints[j].idx_q` (optional),
  `lowerPositionLimit` / `upperPositionLimit`, `frames[f]` (`.name`,
  `.parentJoint` — Pinocchio 3 — or `.parent` — Pinocchio 2 —, `.placement`);
* `cube.model.frames` / `cube.data.oMf` for the hook frames (tools.py:54-59);
* `robot.collision_model` (optional): `geometryObjects[g]` (`.name`,
  `.parentJoint`, `.placement`, `.geometry` with hpp-fcl's attribute names:
  Sphere `.radius`, Box `.halfSide`, Cylinder `.radius` + `.halfLength`, a
  mesh through `.vertices()` / `.num_vertices`) and `collisionPairs[k]`
  (`.first`, `.second`).  The last geometry is the cube that
  `setcubeplacement` moves (tools.py:62-68): it is the solve's target.

The tables are read once per robot object; `computeqgrasppose` caches the
native solver on it.
"""
from __future__ import annotations

import numpy as np

from .collision import BOX, CYLINDER, MESHBOX, SPHERE, CollisionScene, Geom
from .model import DualArmModel, Frame, Joint, KinematicTree, axis_frame

_AXES = {"JointModelRX": 0, "JointModelRY": 1, "JointModelRZ": 2}


def is_pinocchio_like(robot) -> bool:
    m = getattr(robot, "model", None)
    return m is not None and hasattr(m, "jointPlacements") and hasattr(m, "frames")


def _rt(M):
    if hasattr(M, "rotation"):
        return np.array(M.rotation, dtype=np.float64).reshape(3, 3), np.array(M.translation, dtype=np.float64).reshape(3)
    H = np.asarray(M, dtype=np.float64)
    return H[:3, :3].copy(), H[:3, 3].copy()


def _shortname(jm) -> str:
    s = jm.shortname() if callable(getattr(jm, "shortname", None)) else getattr(jm, "shortname", None)
    if s is None:
        raise TypeError(f"joint model {jm!r} has no shortname()")
    return str(s)


def _frame_parent(fr) -> int:
    for attr in ("parentJoint", "parent"):  # Pinocchio 3.x, 2.x
        if hasattr(fr, attr):
            return int(getattr(fr, attr))
    raise TypeError(f"frame {getattr(fr, 'name', fr)!r} has no parentJoint/parent")


def _q_index(model, j: int) -> int:
    jm = model.joints[j]
    iq = getattr(jm, "idx_q", None)
    iq = iq() if callable(iq) else iq
    return int(iq) if iq is not None else j - 1


def tree_from_model(model) -> KinematicTree:
    """KinematicTree (q order) from a Pinocchio Model: revolute joints only,
    one configuration variable each, as the IK kernel requires."""
    nj = int(model.njoints)
    lo = np.asarray(model.lowerPositionLimit, dtype=np.float64)
    hi = np.asarray(model.upperPositionLimit, dtype=np.float64)
    qi = [_q_index(model, j) for j in range(1, nj)]
    if sorted(qi) != list(range(nj - 1)):
        raise ValueError("the IK kernel needs one configuration variable per joint (revolute joints only)")
    slots = [None] * (nj - 1)
    for j in range(1, nj):
        sn = _shortname(model.joints[j])
        if sn in _AXES:
            e = np.zeros(3)
            e[_AXES[sn]] = 1.0
        elif sn == "JointModelRevoluteUnaligned":
            e = np.asarray(model.joints[j].axis, dtype=np.float64).reshape(3)
            e = e / np.linalg.norm(e)
        else:
            raise ValueError(f"joint {model.names[j]}: {sn} is not supported by the IK kernel (revolute only)")
        code, Q = axis_frame(e)
        R, t = _rt(model.jointPlacements[j])
        p = int(model.parents[j])
        k = qi[j - 1]
        slots[k] = Joint(str(model.names[j]), qi[p - 1] if p > 0 else -1, R, t, code, float(lo[k]), float(hi[k]), e, Q)
    tree = KinematicTree(joints=slots)
    for fr in model.frames:
        pj = _frame_parent(fr)
        R, t = _rt(fr.placement)
        tree.frames[str(fr.name)] = Frame(str(fr.name), qi[pj - 1] if pj > 0 else -1, R, t)
    # canonical axes, as parse_urdf does for a URDF
    Qs = [jt.Q for jt in tree.joints]
    for jt in tree.joints:
        Qp = Qs[jt.parent] if jt.parent >= 0 else np.eye(3)
        jt.R, jt.t = Qp.T @ jt.R @ jt.Q, Qp.T @ jt.t
    for f in tree.frames.values():
        if f.parent >= 0:
            f.R, f.t = Qs[f.parent].T @ f.R, Qs[f.parent].T @ f.t
    return tree


def _hook_tree(cube, hooks) -> KinematicTree:
    """The cube's hook frames as tools.getcubeplacement reads them:
    cube.data.oMf[frame id] (framesForwardKinematics at cube.q0, loadobject);
    the frame placements themselves for a jointless model without data."""
    tree = KinematicTree()
    m = cube.model
    names = [str(f.name) for f in m.frames]
    oMf = getattr(getattr(cube, "data", None), "oMf", None)
    for h in hooks:
        if h not in names:
            raise KeyError(f"cube model has no frame {h!r}")
        fid = names.index(h)
        R, t = _rt(oMf[fid] if oMf is not None else m.frames[fid].placement)
        tree.frames[h] = Frame(h, -1, R, t)
    return tree


def model_from_robot(robot, cube, hands=("LARM_EFF", "RARM_EFF"), hooks=("LARM_HOOK", "RARM_HOOK")) -> DualArmModel:
    return DualArmModel.from_trees(tree_from_model(robot.model), _hook_tree(cube, hooks), hands=hands, hooks=hooks)


def _vertices(geom):
    v = getattr(geom, "vertices", None)
    v = v() if callable(v) else v
    if v is None and hasattr(geom, "num_vertices"):
        v = [geom.vertex(i) for i in range(int(geom.num_vertices))]
    if v is None:
        return None
    return np.asarray([np.asarray(x, dtype=np.float64).reshape(3) for x in v])


def _shape(geom):
    """hpp-fcl shape -> (kind, dims, centre offset in the geometry frame)."""
    if type(geom).__name__ in ("Capsule", "Cone", "Ellipsoid", "Plane", "Halfspace"):
        raise ValueError(f"unsupported collision geometry {type(geom).__name__}")
    if hasattr(geom, "halfSide"):
        return BOX, np.asarray(geom.halfSide, dtype=np.float64).reshape(3), np.zeros(3)
    if hasattr(geom, "halfLength") and hasattr(geom, "radius"):
        return CYLINDER, np.array([float(geom.radius), float(geom.halfLength), 0.0]), np.zeros(3)
    if hasattr(geom, "radius"):
        return SPHERE, np.array([float(geom.radius), 0.0, 0.0]), np.zeros(3)
    v = _vertices(geom)
    if v is not None and len(v):
        lo, hi = v.min(axis=0), v.max(axis=0)
        half, ctr = (hi - lo) / 2.0, (hi + lo) / 2.0
        corner = np.abs(np.abs(v - ctr) - half).max()
        if corner > 1e-12 * max(1.0, float(half.max())):
            raise ValueError("mesh geometry is not a box: the kernels model a mesh by its 8-vertex box hull")
        return MESHBOX, half, ctr
    raise ValueError(f"unsupported collision geometry {type(geom).__name__}")


def scene_from_robot(robot, axis_frames=None) -> CollisionScene:
    """CollisionScene from robot.collision_model (setup_pinocchio.py:53-60
    already applied: translaterobot's quirk, the appended table / obstacle /
    cube, the SRDF-filtered pairs plus (46, 47)).  axis_frames: the compiled
    model's joint-frame changes (DualArmModel.axis_frames()); a geometry on a
    joint with a non-canonical axis is re-expressed like the joint's children."""
    cm = robot.collision_model
    model = robot.model
    objs = list(cm.geometryObjects)
    geoms = []
    for k, g in enumerate(objs):
        kind, dims, ctr = _shape(g.geometry)
        R, t = _rt(g.placement)
        pj = int(g.parentJoint)
        target = k == len(objs) - 1  # setcubeplacement moves geometryObjects[-1]
        if target and np.abs(ctr).max() > 0:
            raise ValueError("the cube geometry must be centred on its frame (it is placed at the solve's target)")
        q = _q_index(model, pj) if pj > 0 else -1
        t = t + R @ ctr
        if q >= 0 and axis_frames is not None:
            Qt = np.asarray(axis_frames[q]).T
            R, t = Qt @ R, Qt @ t
        geoms.append(Geom(str(g.name), kind, q, "", R, t, dims, target))
    pairs = np.array([(int(p.first), int(p.second)) for p in cm.collisionPairs], dtype=np.int32).reshape(-1, 2)
    return CollisionScene(geoms, pairs)


def solver_for(robot, cube=None, device: int = 0):
    """The native solver of a foreign robot object, built on first use from
    robot.model, the cube's hook frames and robot.collision_model, and cached
    on the robot per hook set.  Without a cube (collision / distance queries)
    the hooks are identities: any solver already cached serves, since those
    queries never read them."""
    cache = getattr(robot, "_ikgrasp_solvers", None)
    if cache is None:
        cache = {}
        try:
            robot._ikgrasp_solvers = cache
        except AttributeError:  # objects without a __dict__: rebuild per call
            pass
    if cube is None:
        if cache:
            return next(iter(cache.values()))
        hooks = KinematicTree()
        for h in ("LARM_HOOK", "RARM_HOOK"):
            hooks.frames[h] = Frame(h, -1, np.eye(3), np.zeros(3))
        key = None
    else:
        hooks = _hook_tree(cube, ("LARM_HOOK", "RARM_HOOK"))
        key = tuple(np.concatenate([hooks.frames[h].R.ravel().tolist() + hooks.frames[h].t.tolist()
                                    for h in ("LARM_HOOK", "RARM_HOOK")]).tolist())
    s = cache.get(key)
    if s is not None:
        return s
    from .solver import IKSolver
    model = DualArmModel.from_trees(tree_from_model(robot.model), hooks)
    scene = scene_from_robot(robot, model.axis_frames()) if hasattr(robot, "collision_model") else None
    s = IKSolver(model, device=device, scene=scene)
    cache[key] = s
    return s


def target_placement(robot):
    """Where setcubeplacement last put the cube: geometryObjects[-1].placement."""
    R, t = _rt(robot.collision_model.geometryObjects[-1].placement)
    return np.concatenate([R.reshape(9), t])[None, :]
