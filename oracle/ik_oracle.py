"""CPU ORACLE — test infrastructure only, never the product path.

Pure numpy/float64 restatement of the reference grasp-pose IK
(`/root/reference/inverse_geometry.py:17-100`) together with the Pinocchio
semantics it relies on (the reference calls into Pinocchio, which is not
installed in this image; see DESIGN.md "Oracle").  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module, and only as the checker.

Parity status: PINNED.  The oracle reproduces the reference's own golden
outputs KAT-1/KAT-2 (`/root/reference/trajectory.json:3-19` and `:258-274`,
equal bit-for-bit to `trajectory2.json:3-19` / `:326-342`), the joint order
(`lab_instructions.ipynb:210-226`) and the FK pose at q=0
(`lab_instructions.ipynb:290-293`).  The committed fixtures live in
`tests/golden/` (see `tests/golden/make_golden.py`).

The kinematic tables below are transcribed by hand from the URDF so that the
oracle stays independent of the product's URDF model compiler
(`ikgrasp/model.py`); tests check the two agree.
"""
from __future__ import annotations

import math

import numpy as np

# ---------------------------------------------------------------------------
# Model (NextageaOpen.urdf:580-730, setup_pinocchio.py:28-32, config.py:33)
# ---------------------------------------------------------------------------
# q index -> (name, parent q index or -1 for universe, origin xyz, axis 0/1/2, lower, upper)
JOINTS = [
    ("CHEST_JOINT0", -1, (0.0, 0.0, 0.267), 2, -3.14159, 3.14159),          # urdf:580
    ("HEAD_JOINT0", 0, (0.0, 0.0, 0.302), 2, -1.22173, 1.22173),            # urdf:589
    ("HEAD_JOINT1", 1, (0.0, 0.0, 0.08), 1, -0.401425, 1.308997),           # urdf:597
    ("LARM_JOINT0", 0, (0.04, 0.135, 0.1015), 2, -1.5707963, 1.5707963),    # urdf:605
    ("LARM_JOINT1", 3, (0.0, 0.0, 0.066), 1, -2.44346, 1.0471975),          # urdf:614
    ("LARM_JOINT2", 4, (0.0, 0.095, -0.25), 1, -1.22173, 1.5707963),        # urdf:623
    ("LARM_JOINT3", 5, (0.1805, 0.0, -0.03), 0, -3.1415926, 1.7453292),     # urdf:632
    ("LARM_JOINT4", 6, (0.1495, 0.0, 0.0), 1, -3.57792, 1.134464),          # urdf:641
    ("LARM_JOINT5", 7, (0.0, 0.0, -0.1335), 2, -2.7123889, 2.7123889),      # urdf:650
    ("RARM_JOINT0", 0, (0.04, -0.135, 0.1015), 2, -1.570796, 1.570796),     # urdf:659
    ("RARM_JOINT1", 9, (0.0, 0.0, 0.066), 1, -2.44346, 1.047197),           # urdf:668
    ("RARM_JOINT2", 10, (0.0, -0.095, -0.25), 1, -1.22173, 1.570796),       # urdf:677
    ("RARM_JOINT3", 11, (0.1805, 0.0, -0.03), 0, -1.74532, 3.141592),       # urdf:686
    ("RARM_JOINT4", 12, (0.1495, 0.0, 0.0), 1, -3.5779, 1.134464),          # urdf:695
    ("RARM_JOINT5", 13, (0.0, 0.0, -0.1335), 2, -2.712388, 2.712388),       # urdf:704
]
NQ = len(JOINTS)
PARENT = [j[1] for j in JOINTS]
AXIS = [j[3] for j in JOINTS]
LOWER = np.array([j[4] for j in JOINTS])
UPPER = np.array([j[5] for j in JOINTS])
ROBOT_Z = 0.85  # config.py:33 ROBOT_PLACEMENT = XYZQUAT(0,0,0.85, 0,0,0,1)


def urdf_rpy_to_matrix(r: float, p: float, y: float) -> np.ndarray:
    """urdfdom `Rotation::setFromRPY` (+ normalize) followed by Eigen's
    `Quaterniond(w,x,y,z).matrix()` — the path Pinocchio's URDF parser uses to
    turn an `<origin rpy=...>` into a rotation matrix."""
    phi, the, psi = r / 2.0, p / 2.0, y / 2.0
    qx = math.sin(phi) * math.cos(the) * math.cos(psi) - math.cos(phi) * math.sin(the) * math.sin(psi)
    qy = math.cos(phi) * math.sin(the) * math.cos(psi) + math.sin(phi) * math.cos(the) * math.sin(psi)
    qz = math.cos(phi) * math.cos(the) * math.sin(psi) - math.sin(phi) * math.sin(the) * math.cos(psi)
    qw = math.cos(phi) * math.cos(the) * math.cos(psi) + math.sin(phi) * math.sin(the) * math.sin(psi)
    n = math.sqrt(qx * qx + qy * qy + qz * qz + qw * qw)
    qx, qy, qz, qw = qx / n, qy / n, qz / n, qw / n
    tx, ty, tz = 2 * qx, 2 * qy, 2 * qz
    twx, twy, twz = tx * qw, ty * qw, tz * qw
    txx, txy, txz = tx * qx, ty * qx, tz * qx
    tyy, tyz, tzz = ty * qy, tz * qy, tz * qz
    return np.array([
        [1 - (tyy + tzz), txy - twz, txz + twy],
        [txy + twz, 1 - (txx + tzz), tyz - twx],
        [txz - twy, tyz + twx, 1 - (txx + tyy)],
    ])


def joint_placements():
    """Pinocchio `model.jointPlacements[1..15]` after `translaterobot`
    (setup_pinocchio.py:32: jointPlacements[1] = ROBOT_PLACEMENT * jointPlacements[1])."""
    out = []
    for i, (_, _, xyz, _, _, _) in enumerate(JOINTS):
        R = np.eye(3)
        t = np.array(xyz, dtype=np.float64)
        if i == 0:
            t = np.array([0.0, 0.0, ROBOT_Z]) + t  # ROBOT_PLACEMENT (R = I) * placement
        out.append((R, t))
    return out


# Effector frames (NextageaOpen.urdf:717-721, :726-730): parent q index, placement
FRAME_LEFT = (8, urdf_rpy_to_matrix(0.0, 0.0, 1.5708), np.array([0.082, 0.05, -0.02]))
FRAME_RIGHT = (14, urdf_rpy_to_matrix(0.0, 0.0, 1.5708), np.array([0.082, -0.05, -0.02]))
# Cube hook frames (cube_small.urdf:34-37, :44-47)
HOOK_LEFT = (np.eye(3), np.array([0.0, 0.05, 0.0]))
HOOK_RIGHT = (urdf_rpy_to_matrix(0.0, 0.0, -3.14), np.array([0.0, -0.05, 0.0]))

EPSILON = 1e-3  # config.py:22
MAX_ITERS = 1000  # inverse_geometry.py:53
DT = 1e-2  # inverse_geometry.py:54

# ---------------------------------------------------------------------------
# SE3 helpers (Pinocchio conventions: M = (R, p); motion = [linear; angular])
# ---------------------------------------------------------------------------


def se3_mul(A, B):
    Ra, ta = A
    Rb, tb = B
    return (Ra @ Rb, ta + Ra @ tb)


def se3_inv(A):
    R, t = A
    return (R.T, -(R.T @ t))


def axis_rotation(axis: int, q: float) -> np.ndarray:
    """JointModelR{X,Y,Z}::calc — rotation of a revolute joint about a unit axis."""
    s, c = math.sin(q), math.cos(q)
    if axis == 0:
        return np.array([[1.0, 0.0, 0.0], [0.0, c, -s], [0.0, s, c]])
    if axis == 1:
        return np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])
    return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])


def forward_kinematics(q, placements=None):
    """pin.forwardKinematics: oMi[j] = oMi[parent] * (jointPlacement_j * jMi(q_j))."""
    placements = placements or joint_placements()
    oMi = []
    for j in range(NQ):
        R0, t0 = placements[j]
        liMi = (R0 @ axis_rotation(AXIS[j], q[j]), t0.copy())
        oMi.append(liMi if PARENT[j] < 0 else se3_mul(oMi[PARENT[j]], liMi))
    return oMi


def frame_placement(oMi, frame):
    """pin.updateFramePlacements: oMf = oMi[frame.parent] * frame.placement."""
    j, R, t = frame
    return se3_mul(oMi[j], (R, t))


def log3(R):
    """pin.log3 (Pinocchio spatial/explog.hpp, 2.6-era branch structure)."""
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 3.0:
        theta = 0.0
    elif tr < -1.0:
        theta = math.pi
    else:
        theta = math.acos((tr - 1.0) / 2.0)
    if theta >= math.pi - 1e-2:
        cphi = math.cos(theta - math.pi)
        beta = theta * theta / (1.0 + cphi)
        tmp = (np.diag(R) + cphi) * beta
        w = np.empty(3)
        w[0] = (1.0 if R[2, 1] > R[1, 2] else -1.0) * (math.sqrt(tmp[0]) if tmp[0] > 0 else 0.0)
        w[1] = (1.0 if R[0, 2] > R[2, 0] else -1.0) * (math.sqrt(tmp[1]) if tmp[1] > 0 else 0.0)
        w[2] = (1.0 if R[1, 0] > R[0, 1] else -1.0) * (math.sqrt(tmp[2]) if tmp[2] > 0 else 0.0)
    else:
        prec3 = np.finfo(np.float64).eps ** 0.25  # TaylorSeriesExpansion::precision<3>()
        t = (theta / math.sin(theta) if theta > prec3 else 1.0) / 2.0
        w = np.array([t * (R[2, 1] - R[1, 2]), t * (R[0, 2] - R[2, 0]), t * (R[1, 0] - R[0, 1])])
    return w, theta


def log6(M):
    """pin.log6 -> 6-vector [v; w]."""
    R, p = M
    w, t = log3(R)
    t2 = t * t
    prec3 = np.finfo(np.float64).eps ** 0.25
    if t < prec3:
        alpha = 1.0 - t2 / 12.0 - t2 * t2 / 720.0
        beta = 1.0 / 12.0 + t2 / 720.0
    else:
        st, ct = math.sin(t), math.cos(t)
        alpha = t * st / (2.0 * (1.0 - ct))
        beta = 1.0 / t2 - st / (2.0 * t * (1.0 - ct))
    v = alpha * p - 0.5 * np.cross(w, p) + (beta * np.dot(w, p)) * w
    return np.concatenate([v, w])


def frame_jacobian_local(q, frame, placements=None):
    """pin.computeFrameJacobian(model, data, q, fid) with the default LOCAL frame:
    backward pass over the frame's support, col_i = iMf.actInv(S_i),
    iMf <- liMi * iMf."""
    placements = placements or joint_placements()
    j, Rf, tf = frame
    J = np.zeros((6, NQ))
    iMf = (Rf.copy(), tf.copy())
    i = j
    while i >= 0:
        R, t = iMf
        a = np.zeros(3)
        a[AXIS[i]] = 1.0
        J[:3, i] = R.T @ (-np.cross(t, a))
        J[3:, i] = R.T @ a
        R0, t0 = placements[i]
        liMi = (R0 @ axis_rotation(AXIS[i], q[i]), t0)
        iMf = se3_mul(liMi, iMf)
        i = PARENT[i]
    return J


def hook_targets(cube_R, cube_t):
    """tools.getcubeplacement: oMcube * cube.data.oMf[hook] (tools.py:54-59)."""
    M = (np.asarray(cube_R, dtype=np.float64), np.asarray(cube_t, dtype=np.float64))
    return se3_mul(M, HOOK_LEFT), se3_mul(M, HOOK_RIGHT)


def hand_errors(q, oMcubeL, oMcubeR, placements=None):
    oMi = forward_kinematics(q, placements)
    oMhL = frame_placement(oMi, FRAME_LEFT)
    oMhR = frame_placement(oMi, FRAME_RIGHT)
    eL = log6(se3_mul(se3_inv(oMhL), oMcubeL))
    eR = log6(se3_mul(se3_inv(oMhR), oMcubeR))
    return eL, eR


def pinv_exact(J, e, dps=40):
    """pinv(J) e evaluated in dps-digit arithmetic on the float64 J and e, with
    np.linalg.pinv's cut (singular values below 1e-15 sigma_max dropped), then
    rounded to float64.  For the fixtures at arm singularities: where J is
    ill-conditioned, np.linalg.pinv's own result carries ~eps * cond(J) of
    LAPACK rounding (at cond(J) = 1.8e10 it puts 79 rad into the exactly-zero
    head columns on the first step, tools/singular_probe.py); this is the
    value it approximates.  Rank decisions come from a 40-digit SVD when
    numpy's sigma_min / sigma_max < 1e-13, else the normal equations suffice
    (cond(J)^2 << 10^dps)."""
    import mpmath as mp
    mp.mp.dps = dps
    s = np.linalg.svd(J, compute_uv=False)
    Jm = mp.matrix(J.tolist())
    em = mp.matrix(list(map(float, e)))
    if s[-1] < 1e-13 * s[0]:
        U, S, V = mp.svd_r(Jm)
        cut = mp.mpf("1e-15") * S[0]
        x = mp.matrix(J.shape[1], 1)
        for i in range(len(S)):
            if S[i] > cut:
                ui = U[:, i]
                x += V[i, :].T * ((ui.T * em)[0] / S[i])
    else:
        x = Jm.T * mp.lu_solve(Jm * Jm.T, em)
    return np.array([float(v) for v in x])


def computeqgrasppose(q0, cube_R, cube_t, max_iters=MAX_ITERS, dt=DT, eps=EPSILON, lam=0.0, step=None):
    """Restatement of inverse_geometry.py:41-100 without the collision term.

    Returns (q, converged, iters, (|eL|, |eR|)) where `iters` is the number of
    joint updates applied (== index of the converged check).  `lam > 0`
    replaces pinv(J) e by J^T (J J^T + lam I)^-1 e — an extension the
    reference does not have (parity for it is unpinned).  `step(J, e)`
    replaces np.linalg.pinv(J) @ e (e.g. pinv_exact).
    """
    placements = joint_placements()
    oMcubeL, oMcubeR = hook_targets(cube_R, cube_t)
    q = np.array(q0, dtype=np.float64).copy()  # :49
    for it in range(max_iters):  # :56
        eL, eR = hand_errors(q, oMcubeL, oMcubeR, placements)  # :58-67
        nL, nR = np.linalg.norm(eL), np.linalg.norm(eR)
        if nL < eps and nR < eps:  # :70 (collision term: out of scope)
            return q, True, it, (nL, nR)
        JL = frame_jacobian_local(q, FRAME_LEFT, placements)  # :75
        JR = frame_jacobian_local(q, FRAME_RIGHT, placements)  # :76
        e = np.hstack([eL, eR])  # :79
        J = np.vstack([JL, JR])  # :80
        if lam > 0:
            vq = J.T @ np.linalg.solve(J @ J.T + lam * np.eye(12), e)
        elif step is not None:
            vq = step(J, e)
        else:
            vq = np.linalg.pinv(J) @ e  # :83
        q = q + vq * dt  # :86 pin.integrate on revolute joints
        q = np.minimum(np.maximum(LOWER, q), UPPER)  # :89 tools.py:21-22
    eL, eR = hand_errors(q, oMcubeL, oMcubeR, placements)
    return q, False, max_iters, (np.linalg.norm(eL), np.linalg.norm(eR))


def computeqgrasppose_mp(q0, cube_R, cube_t, dps=32, max_iters=MAX_ITERS, dt=DT, eps=EPSILON):
    """The loop of `computeqgrasppose` evaluated in `dps`-digit arithmetic
    (mpmath) from the float64 model constants and inputs, rounded to float64
    only at the end: the mathematically exact answer the float64 loops
    approximate.  Where a trajectory is sensitive (random seeds, a slow
    approach), the reference's own float64 result carries rounding noise of
    ~1e-8 (its acos((tr-1)/2) near theta ~1e-3 loses ~10 digits), so this, not
    one float64 run, is what "within 1e-9" is measured against
    (tests/golden/sensitive_cases.npz).  Slow (~0.1 s per update)."""
    import mpmath as mp
    mp.mp.dps = dps
    f = mp.mpf
    pl = joint_placements()

    def mat(A):
        return [[f(float(A[i][j])) for j in range(3)] for i in range(3)]

    def vec(v):
        return [f(float(x)) for x in v]

    def mm(A, B):
        return [[A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j] for j in range(3)] for i in range(3)]

    def mv(A, v):
        return [A[i][0] * v[0] + A[i][1] * v[1] + A[i][2] * v[2] for i in range(3)]

    def mtv(A, v):
        return [A[0][i] * v[0] + A[1][i] * v[1] + A[2][i] * v[2] for i in range(3)]

    def tr(A):
        return [[A[j][i] for j in range(3)] for i in range(3)]

    def rot(axis, q):
        s, c = mp.sin(q), mp.cos(q)
        o, z = f(1), f(0)
        if axis == 0:
            return [[o, z, z], [z, c, -s], [z, s, c]]
        if axis == 1:
            return [[c, z, s], [z, o, z], [-s, z, c]]
        return [[c, -s, z], [s, c, z], [z, z, o]]

    def se3(A, B):
        return (mm(A[0], B[0]), [A[1][i] + mv(A[0], B[1])[i] for i in range(3)])

    P = [(mat(R0), vec(t0)) for R0, t0 in pl]
    frames = [(j, mat(Rf), vec(tf)) for j, Rf, tf in (FRAME_LEFT, FRAME_RIGHT)]
    cube = (mat(cube_R), vec(cube_t))
    tgts = [se3(cube, (mat(H[0]), vec(H[1]))) for H in (HOOK_LEFT, HOOK_RIGHT)]
    lo, hi = [f(float(x)) for x in LOWER], [f(float(x)) for x in UPPER]

    def log6_mp(R, p):
        sk = [R[2][1] - R[1][2], R[0][2] - R[2][0], R[1][0] - R[0][1]]
        s = mp.sqrt(sk[0] ** 2 + sk[1] ** 2 + sk[2] ** 2) / 2
        c = (R[0][0] + R[1][1] + R[2][2] - 1) / 2
        th = mp.atan2(s, c)
        if th >= mp.pi - f("1e-2"):
            cphi = -c
            b = th * th / (1 + cphi)
            w = []
            for i, (a_, b_) in enumerate(((2, 1), (0, 2), (1, 0))):
                tmp = (R[i][i] + cphi) * b
                sg = 1 if R[a_][b_] > R[b_][a_] else -1
                w.append(sg * (mp.sqrt(tmp) if tmp > 0 else f(0)))
        else:
            k = th / (2 * s) if s > 0 else f("0.5")
            w = [k * x for x in sk]
        if th == 0:
            al, be = f(1), f(1) / 12
        else:
            al = th * mp.sin(th) / (2 * (1 - mp.cos(th)))
            be = 1 / (th * th) - mp.sin(th) / (2 * th * (1 - mp.cos(th)))
        wp = w[0] * p[0] + w[1] * p[1] + w[2] * p[2]
        cr = [w[1] * p[2] - w[2] * p[1], w[2] * p[0] - w[0] * p[2], w[0] * p[1] - w[1] * p[0]]
        return [al * p[i] - cr[i] / 2 + be * wp * w[i] for i in range(3)] + w

    q = [f(float(x)) for x in q0]
    for it in range(max_iters + 1):
        oMi = []
        for j in range(NQ):
            l = (mm(P[j][0], rot(AXIS[j], q[j])), P[j][1])
            oMi.append(l if PARENT[j] < 0 else se3(oMi[PARENT[j]], l))
        es, Js = [], []
        for h, (j, Rf, tf) in enumerate(frames):
            Rh, th_ = se3(oMi[j], (Rf, tf))
            TR, Tt = tgts[h]
            es.append(log6_mp(mm(tr(Rh), TR), mtv(Rh, [Tt[i] - th_[i] for i in range(3)])))
            J = [[f(0)] * NQ for _ in range(6)]
            i = j
            while i >= 0:  # LOCAL: column = [R_f^T (a x (p_f - o_i)); R_f^T a]
                a = [oMi[i][0][r][AXIS[i]] for r in range(3)]
                d = [th_[r] - oMi[i][1][r] for r in range(3)]
                cr = [a[1] * d[2] - a[2] * d[1], a[2] * d[0] - a[0] * d[2], a[0] * d[1] - a[1] * d[0]]
                lin, ang = mtv(Rh, cr), mtv(Rh, a)
                for r in range(3):
                    J[r][i], J[3 + r][i] = lin[r], ang[r]
                i = PARENT[i]
            Js.append(J)
        nL = mp.sqrt(sum(x * x for x in es[0]))
        nR = mp.sqrt(sum(x * x for x in es[1]))
        if it >= max_iters or (nL < eps and nR < eps):
            break
        Jm = mp.matrix(Js[0] + Js[1])
        em = mp.matrix(es[0] + es[1])
        x = Jm.T * mp.lu_solve(Jm * Jm.T, em)
        q = [min(max(lo[k], q[k] + x[k] * f(dt)), hi[k]) for k in range(NQ)]
    conv = bool(nL < eps and nR < eps) and it < max_iters
    return np.array([float(v) for v in q]), conv, it, (float(nL), float(nR))


def fk_hands(q):
    """(oMhandL, oMhandR) at q — used by tests for EE-space comparisons."""
    oMi = forward_kinematics(np.asarray(q, dtype=np.float64))
    return frame_placement(oMi, FRAME_LEFT), frame_placement(oMi, FRAME_RIGHT)
