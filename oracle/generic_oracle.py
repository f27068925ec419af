"""CPU ORACLE — test infrastructure only, never the product path.

Generic-chain restatement of the grasp-pose IK (`/root/reference/
inverse_geometry.py:41-100`) for the model-generality row:
any URDF tree of revolute + fixed joints, any joint axis direction (Pinocchio's
RX/RY/RZ for +X/+Y/+Z and RevoluteUnaligned, rotation exp(q [e]x) about the
normalised axis, otherwise).  It reads the URDF itself and works in the raw
joint frames with Rodrigues rotations, so it is independent of the product's
model compiler (`ikgrasp/model.py`), which instead re-expresses
non-canonical axes onto X/Y/Z.

Same loop as `ik_oracle.computeqgrasppose`: FK, log6 errors of the two hands
against the cube's hooks, LOCAL frame Jacobians, `np.linalg.pinv(J) @ e`,
q + dt vq, clip to the limits (the collision term is not modelled here).

Parity status: pinned through the Nextage KATs — on the reference's own URDF
this restatement reproduces KAT-1/KAT-2 (`trajectory.json:3-19`, `:258-274`)
in 740 / 736 iterations (`tests/test_generic_model.py`, when the reference
tree is present; the check also runs in `tests/golden/make_golden.py
generic`).  For other robots (the synthetic tilted-axis robot in
`tests/golden/`) no reference outputs exist: the oracle is the statement of
Pinocchio's semantics above.
"""
from __future__ import annotations

import math
import os
import xml.etree.ElementTree as ET

import numpy as np

from oracle import ik_oracle as ik


def _floats(s, n, default):
    if s is None:
        return np.array(default, dtype=np.float64)
    v = [float(t) for t in s.split()]
    assert len(v) == n, s
    return np.array(v)


def _origin(el):
    o = el.find("origin")
    xyz = _floats(o.get("xyz") if o is not None else None, 3, (0.0, 0.0, 0.0))
    rpy = _floats(o.get("rpy") if o is not None else None, 3, (0.0, 0.0, 0.0))
    return ik.urdf_rpy_to_matrix(*rpy), xyz


def rodrigues(e, q):
    """exp(q [e]x) for a unit axis e (JointModelRevoluteUnaligned::calc)."""
    s, c = math.sin(q), math.cos(q)
    K = np.array([[0.0, -e[2], e[1]], [e[2], 0.0, -e[0]], [-e[1], e[0], 0.0]])
    return np.eye(3) + s * K + (1.0 - c) * (K @ K)


class ChainModel:
    """Joints in Pinocchio order (depth first, siblings by joint name), fixed
    joints folded into frames and into the next joint's placement."""

    def __init__(self, urdf, base_placement=None):
        root = ET.parse(urdf).getroot() if os.path.exists(urdf) else ET.fromstring(urdf)
        links = {l.get("name") for l in root.findall("link")}
        kids, child_links = {}, set()
        for j in root.findall("joint"):
            kids.setdefault(j.find("parent").get("link"), []).append(j)
            child_links.add(j.find("child").get("link"))
        (root_link,) = sorted(links - child_links)
        self.names, self.parent, self.placement, self.axis, self.lower, self.upper = [], [], [], [], [], []
        self.frames = {root_link: (-1, (np.eye(3), np.zeros(3)))}
        self.link_frame = {root_link: (-1, (np.eye(3), np.zeros(3)))}
        self.urdf_root = root

        def visit(link, pj, M):
            for j in sorted(kids.get(link, []), key=lambda e: e.get("name")):
                child = j.find("child").get("link")
                O = ik.se3_mul(M, _origin(j))
                if j.get("type") == "fixed":
                    self.frames[j.get("name")] = (pj, O)
                    self.link_frame[child] = (pj, O)
                    visit(child, pj, O)
                elif j.get("type") == "revolute":
                    if pj < 0 and base_placement is not None:
                        O = ik.se3_mul(base_placement, O)
                    a = _floats(j.find("axis").get("xyz") if j.find("axis") is not None else None, 3, (1, 0, 0))
                    lim = j.find("limit")
                    self.names.append(j.get("name"))
                    self.parent.append(pj)
                    self.placement.append(O)
                    self.axis.append(a / np.linalg.norm(a))
                    self.lower.append(float(lim.get("lower", "0")) if lim is not None else 0.0)
                    self.upper.append(float(lim.get("upper", "0")) if lim is not None else 0.0)
                    idx = len(self.names) - 1
                    I0 = (np.eye(3), np.zeros(3))
                    self.frames[j.get("name")] = (idx, I0)
                    self.link_frame[child] = (idx, I0)
                    visit(child, idx, I0)
                else:
                    raise ValueError(f"joint type {j.get('type')} not modelled")

        visit(root_link, -1, (np.eye(3), np.zeros(3)))
        self.nq = len(self.names)
        self.lower = np.array(self.lower)
        self.upper = np.array(self.upper)

    def fk(self, q):
        oMi = []
        for j in range(self.nq):
            R0, t0 = self.placement[j]
            liMi = (R0 @ rodrigues(self.axis[j], q[j]), t0.copy())
            oMi.append(liMi if self.parent[j] < 0 else ik.se3_mul(oMi[self.parent[j]], liMi))
        return oMi

    def frame(self, oMi, name):
        j, M = self.frames[name]
        return M if j < 0 else ik.se3_mul(oMi[j], M)

    def frame_jacobian_local(self, q, name, oMi=None):
        """computeFrameJacobian (LOCAL): column i over the support = [R_f^T (a_i x (p_f - o_i)); R_f^T a_i]."""
        oMi = oMi if oMi is not None else self.fk(q)
        Rf, pf = self.frame(oMi, name)
        J = np.zeros((6, self.nq))
        i = self.frames[name][0]
        while i >= 0:
            Ri, oi = oMi[i]
            a = Ri @ self.axis[i]
            J[:3, i] = Rf.T @ np.cross(a, pf - oi)
            J[3:, i] = Rf.T @ a
            i = self.parent[i]
        return J

    def geometry_placements(self, oMi):
        """World placement of every <collision> of every link (link order of the URDF)."""
        out = {}
        for link in self.urdf_root.findall("link"):
            j, M = self.link_frame[link.get("name")]
            for k, c in enumerate(link.findall("collision")):
                G = ik.se3_mul(M, _origin(c))
                out[f"{link.get('name')}_{k}"] = G if j < 0 else ik.se3_mul(oMi[j], G)
        return out


def cube_hooks(cube_urdf, hooks=("LARM_HOOK", "RARM_HOOK")):
    c = ChainModel(cube_urdf)
    return [c.frames[h][1] for h in hooks]


def computeqgrasppose(model, hooks, q0, cube_R, cube_t, hands=("LARM_EFF", "RARM_EFF"), max_iters=ik.MAX_ITERS,
                      dt=ik.DT, eps=ik.EPSILON):
    """inverse_geometry.py:41-100 on a generic model (no collision term).
    Returns (q, converged, updates, (|eL|, |eR|))."""
    cube = (np.asarray(cube_R, dtype=np.float64), np.asarray(cube_t, dtype=np.float64))
    targets = [ik.se3_mul(cube, hk) for hk in hooks]
    q = np.array(q0, dtype=np.float64).copy()

    def errors(q):
        oMi = model.fk(q)
        es = [ik.log6(ik.se3_mul(ik.se3_inv(model.frame(oMi, h)), T)) for h, T in zip(hands, targets)]
        return oMi, es

    for it in range(max_iters):
        oMi, (eL, eR) = errors(q)
        nL, nR = np.linalg.norm(eL), np.linalg.norm(eR)
        if nL < eps and nR < eps:
            return q, True, it, (nL, nR)
        J = np.vstack([model.frame_jacobian_local(q, h, oMi) for h in hands])
        vq = np.linalg.pinv(J) @ np.hstack([eL, eR])
        q = np.minimum(np.maximum(model.lower, q + vq * dt), model.upper)
    _, (eL, eR) = errors(q)
    return q, False, max_iters, (np.linalg.norm(eL), np.linalg.norm(eR))
