"""Round 3 probe: the kernel arithmetic (host emulator) against the numpy
pinv oracle from seeds at and near the arm-block singularities:
wrist (arm joint 4 at -pi/2: c4 = 0), straight elbow (det2 = 0) and
shoulder (wrist centre on arm joint 0's axis: w_x = 0)."""
import ctypes as C
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "motion-planning-and-control-for-dual-manipulator-robot_amd")]
from ikgrasp import _lib  # noqa: E402
from ikgrasp.model import load_nextage  # noqa: E402
from ikgrasp.workload import uniform_targets  # noqa: E402
from oracle import ik_oracle as O  # noqa: E402

lib = C.CDLL(os.path.join(os.path.dirname(_lib.LIB_PATH), "libikgrasp_emu.so"))
vp = C.c_void_p
lib.ikg_emu_solve.argtypes = [vp, C.c_int, vp, vp, C.c_int64, C.c_int64, vp, vp, vp, vp, vp, vp, C.c_int, vp]
lib.ikg_emu_lq_count.restype = C.c_longlong
lib.ikg_emu_svd_count.restype = C.c_longlong
desc = _lib.model_desc(load_nextage())


def emu(tg, q0, dtype=0):
    B = len(tg)
    npt = np.float64 if dtype == 0 else np.float32
    q0 = np.ascontiguousarray(q0, dtype=npt)
    p = _lib.default_params()
    q = np.empty((B, 15), npt); conv = np.empty(B, np.uint8); it = np.empty(B, np.int32); err = np.empty((B, 2), npt)
    lib.ikg_emu_solve(C.byref(desc), dtype, np.ascontiguousarray(tg, dtype=npt).ctypes.data, q0.ctypes.data, 15, B, C.byref(p),
                      q.ctypes.data, conv.ctypes.data, it.ctypes.data, err.ctypes.data, None, 0, None)
    return q, conv.astype(bool), it


def blocks(q):
    tg = uniform_targets(1, seed=0)[0]
    oL, oR = O.hook_targets(tg[:9].reshape(3, 3), tg[9:])
    JL = O.frame_jacobian_local(q, O.FRAME_LEFT)
    JR = O.frame_jacobian_local(q, O.FRAME_RIGHT)
    J = np.vstack([JL, JR])
    s = np.linalg.svd(J, compute_uv=False)
    return s[0] / s[-1], 1.0 / np.linalg.svd(JL[:, 3:9], compute_uv=False)[-1]


def main():
    rng = np.random.default_rng(7)
    cases = []
    for d in (0.0, 1e-9, 1e-6, 1e-3):
        for arm, j in (("L", 7), ("R", 13)):
            q = np.zeros(15)
            q[j] = -math.pi / 2 + d
            cases.append((f"wrist {arm} -pi/2{d:+.0e}", q))
    # straight elbow (det2 = 0) and shoulder (w_x = 0), found by root finding
    # on the frame-1 geometry (all other joints 0): LARM/RARM_JOINT2 and _JOINT1
    for d in (0.0, 1e-9, 1e-6, 1e-3):
        for arm, j, v in (("L", 5, 1.4801364395941514), ("R", 11, 1.4801364395941514),
                          ("L", 4, 0.8671825440154443), ("R", 10, -2.2744101095743487)):
            q = np.zeros(15)
            q[j] = v + d
            cases.append((f"{'elbow' if j in (5, 11) else 'shoulder'} {arm} {d:+.0e}", q))
    tg = uniform_targets(len(cases), seed=11)
    for (name, q), t in zip(cases, tg):
        kJ, kA = blocks(q)
        qo, co, io, _ = O.computeqgrasppose(q, t[:9].reshape(3, 3), t[9:])
        lib.ikg_emu_lq_count(1)
        qe, ce, ie = emu(t[None], q[None])
        nlq = f"{lib.ikg_emu_lq_count(1)}/{lib.ikg_emu_svd_count(1)}"
        q32, c32, i32 = emu(t[None], q[None], dtype=1)
        nlq32 = lib.ikg_emu_lq_count(1)
        print(f"{name:28s} cond(J)={kJ:9.2e} |J_L^-1|={kA:9.2e} oracle conv={co} it={io:4d} | "
              f"emu conv={bool(ce[0])} it={ie[0]:4d} |dq|={np.abs(qe[0]-qo).max():.2e} lq={nlq} | "
              f"f32 conv={bool(c32[0])} it={i32[0]:4d} |dq|={np.abs(q32[0]-qo).max():.1e} lq={nlq32}", flush=True)


if __name__ == "__main__":
    main()
