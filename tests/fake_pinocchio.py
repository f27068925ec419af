"""Plain-Python stand-ins for the reference's Pinocchio objects (test
infrastructure): a RobotWrapper-shaped `robot` and `cube` carrying exactly
the attributes /root/reference/setup_pinocchio.py:73-83 leaves on them and
ikgrasp.pinocchio_bridge reads (model.jointPlacements, joints[j].shortname(),
frames, limits, collision_model.geometryObjects / collisionPairs with
hpp-fcl-named shape attributes).  They are filled from the compiled Nextage
tables and scene, the way a Pinocchio build of the same URDFs is laid out:
universe = joint 0, q index = joint id - 1."""
import numpy as np


class SE3:
    def __init__(self, R, t):
        self.rotation = np.array(R, dtype=np.float64)
        self.translation = np.array(t, dtype=np.float64)


class JointModel:
    def __init__(self, short, idx_q):
        self._short = short
        self.idx_q = idx_q

    def shortname(self):
        return self._short


class Frame:
    def __init__(self, name, parent_joint, placement, pin2=False):
        self.name = name
        self.placement = placement
        if pin2:
            self.parent = parent_joint  # Pinocchio 2.x spelling
        else:
            self.parentJoint = parent_joint


class Box:
    def __init__(self, half):
        self.halfSide = np.array(half, dtype=np.float64)


class Cylinder:
    def __init__(self, r, hl):
        self.radius, self.halfLength = float(r), float(hl)


class Sphere:
    def __init__(self, r):
        self.radius = float(r)


class Mesh:  # a BVHModel: vertices() only
    def __init__(self, half):
        h = np.asarray(half, dtype=np.float64)
        self._v = np.array([[sx * h[0], sy * h[1], sz * h[2]] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])

    def vertices(self):
        return self._v


class GeometryObject:
    def __init__(self, name, parent_joint, placement, geometry):
        self.name, self.parentJoint, self.placement, self.geometry = name, parent_joint, placement, geometry


class Pair:
    def __init__(self, a, b):
        self.first, self.second = int(a), int(b)


class NS:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def nextage_wrapper(pin2=False):
    """(robot, cube) shaped like setuppinocchio()'s, from the compiled tables."""
    from ikgrasp.collision import BOX, CYLINDER, MESHBOX, SPHERE, load_nextage_scene
    from ikgrasp.model import load_nextage
    m = load_nextage()
    scene = load_nextage_scene()
    nq = m.nq
    axes = {0: "JointModelRX", 1: "JointModelRY", 2: "JointModelRZ"}
    joints = [JointModel("JointModelFreeFlyer-unused", -1)] + [JointModel(axes[int(m.axis[k])], k) for k in range(nq)]
    placements = [SE3(np.eye(3), np.zeros(3))] + [SE3(m.R[k], m.t[k]) for k in range(nq)]
    parents = [0] + [p + 1 for p in m.parents]
    frames = [Frame("universe", 0, SE3(np.eye(3), np.zeros(3)), pin2)]
    frames += [Frame(n, k + 1, SE3(np.eye(3), np.zeros(3)), pin2) for k, n in enumerate(m.joint_names)]
    last = [int(m.arm_q[a][-1]) for a in range(2)]
    frames += [Frame(m.hand_names[a], last[a] + 1, SE3(m.hand_R[a], m.hand_t[a]), pin2) for a in range(2)]
    model = NS(njoints=nq + 1, names=["universe"] + list(m.joint_names), parents=parents,
               jointPlacements=placements, joints=joints, frames=frames,
               lowerPositionLimit=m.lower.copy(), upperPositionLimit=m.upper.copy(), nq=nq)
    shape = {SPHERE: lambda d: Sphere(d[0]), BOX: lambda d: Box(d), CYLINDER: lambda d: Cylinder(d[0], d[1]),
             MESHBOX: lambda d: Mesh(d)}
    geoms = [GeometryObject(g.name, g.joint + 1, SE3(g.R, g.t), shape[g.kind](g.dims)) for g in scene.geoms]
    robot = NS(model=model, collision_model=NS(geometryObjects=geoms, collisionPairs=[Pair(a, b) for a, b in scene.pairs]),
               visual_model=NS(geometryObjects=[GeometryObject(g.name, g.parentJoint, g.placement, None) for g in geoms]),
               q0=np.zeros(nq))
    cube_frames = [Frame("universe", 0, SE3(np.eye(3), np.zeros(3)), pin2)]
    cube_frames += [Frame(h, 0, SE3(m.hook_R[a], m.hook_t[a]), pin2) for a, h in enumerate(m.hook_names)]
    cube_geom = GeometryObject("cube_0", 0, SE3(np.eye(3), np.zeros(3)), Mesh(scene.geoms[-1].dims))
    cube = NS(model=NS(frames=cube_frames), data=NS(oMf=[f.placement for f in cube_frames]),
              collision_model=NS(geometryObjects=[cube_geom]),
              visual_model=NS(geometryObjects=[GeometryObject("cube_0", 0, cube_geom.placement, None)]),
              q0=np.zeros(0))
    return robot, cube
