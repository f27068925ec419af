"""ctypes loader for the C oracle (oracle/ikg_oracle.c) — test/baseline
infrastructure only (tests/, smoke(), bench.py cpu_baseline)."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("IKG_ORACLE_LIB", os.path.join(HERE, "_build", "libikg_oracle.so"))
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise FileNotFoundError(f"{LIB} missing: run `make -C oracle` or __graft_entry__.build()")
        lib = C.CDLL(LIB)
        lib.ikg_oracle_solve.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_double,
                                         C.c_double, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        lib.ikg_oracle_solve.restype = C.c_int
        lib.ikg_oracle_max_threads.restype = C.c_int
        _lib = lib
    return _lib


def solve(targets, q0, max_iters=1000, eps=1e-3, dt=1e-2, threads=0):
    tg = np.ascontiguousarray(targets, dtype=np.float64).reshape(-1, 12)
    B = tg.shape[0]
    q = np.ascontiguousarray(q0, dtype=np.float64)
    stride = 0 if q.ndim == 1 else 15
    q_out = np.empty((B, 15))
    conv = np.empty(B, dtype=np.uint8)
    iters = np.empty(B, dtype=np.int32)
    err = np.empty((B, 2))
    load().ikg_oracle_solve(tg.ctypes.data, q.ctypes.data, stride, B, max_iters, eps, dt, q_out.ctypes.data,
                            conv.ctypes.data, iters.ctypes.data, err.ctypes.data, threads)
    return q_out, conv.astype(bool), iters, err


# evaluation options of ikg_oracle_solve_ex (oracle/ikg_oracle.c, orc_opts)
ACC_LOG6 = 1  # log3/log6 without the reference's acos((tr-1)/2) / 1-cos cancellation
QR_STEP = 2   # pinv(J) e by Householder QR of J^T (np.linalg.pinv's error class)
JITTER = 4    # every FK rotation entry moved by 0 / +-1 ulp: the reference's own rounding envelope


def solve_ex(targets, q0, flags=0, seed=0, first=0, max_iters=1000, eps=1e-3, dt=1e-2, threads=0):
    """`solve` with evaluation options (flags above; `seed` keys the jitter,
    `first` is the problem index of row 0 so a subset reproduces a run)."""
    lib = load()
    f = lib.ikg_oracle_solve_ex
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_double, C.c_double, C.c_int,
                  C.c_uint64, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    f.restype = C.c_int
    tg = np.ascontiguousarray(targets, dtype=np.float64).reshape(-1, 12)
    B = tg.shape[0]
    q = np.ascontiguousarray(q0, dtype=np.float64)
    stride = 0 if q.ndim == 1 else 15
    q_out = np.empty((B, 15))
    conv = np.empty(B, dtype=np.uint8)
    iters = np.empty(B, dtype=np.int32)
    err = np.empty((B, 2))
    f(tg.ctypes.data, q.ctypes.data, stride, B, max_iters, eps, dt, flags, seed, first, q_out.ctypes.data,
      conv.ctypes.data, iters.ctypes.data, err.ctypes.data, threads)
    return q_out, conv.astype(bool), iters, err


def has_collision():
    """The C restatement of the collision term (ikg_oracle_solve_collision) is built in."""
    return hasattr(load(), "ikg_oracle_solve_collision")


def _scene_arrays(scene):
    """collision_oracle scene (dict from load_scene / prepare) -> the C arrays."""
    gs = scene["geoms"]
    a = dict(
        kind=np.ascontiguousarray([g["kind"] for g in gs], dtype=np.int32),
        joint=np.ascontiguousarray([g["joint"] for g in gs], dtype=np.int32),
        R=np.ascontiguousarray([np.asarray(g["R"], dtype=np.float64).reshape(9) for g in gs]),
        t=np.ascontiguousarray([np.asarray(g["t"], dtype=np.float64).reshape(3) for g in gs]),
        dims=np.ascontiguousarray([np.asarray(g["dims"], dtype=np.float64).reshape(3) for g in gs]),
        target=np.ascontiguousarray([bool(g["target"]) for g in gs], dtype=np.uint8),
        pairs=np.ascontiguousarray(np.asarray(scene["pairs"], dtype=np.int32).reshape(-1, 2)),
    )
    return a


def _scene_args(a):
    return [len(a["kind"]), a["kind"].ctypes.data, a["joint"].ctypes.data, a["R"].ctypes.data, a["t"].ctypes.data,
            a["dims"].ctypes.data, a["target"].ctypes.data, len(a["pairs"]), a["pairs"].ctypes.data]


_SCENE_T = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]


def solve_collision(scene, targets, q0, max_iters=1000, eps=1e-3, dt=1e-2, threads=0):
    """computeqgrasppose WITH the collision term (inverse_geometry.py:70, :97-98),
    restating collision_oracle.computeqgrasppose in C."""
    lib = load()
    f = lib.ikg_oracle_solve_collision
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int, C.c_double, C.c_double] + _SCENE_T + \
        [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    f.restype = C.c_int
    a = _scene_arrays(scene)
    tg = np.ascontiguousarray(targets, dtype=np.float64).reshape(-1, 12)
    B = tg.shape[0]
    q = np.ascontiguousarray(q0, dtype=np.float64)
    stride = 0 if q.ndim == 1 else 15
    q_out = np.empty((B, 15))
    conv = np.empty(B, dtype=np.uint8)
    iters = np.empty(B, dtype=np.int32)
    err = np.empty((B, 2))
    rc = f(tg.ctypes.data, q.ctypes.data, stride, B, max_iters, eps, dt, *_scene_args(a), q_out.ctypes.data,
           conv.ctypes.data, iters.ctypes.data, err.ctypes.data, threads)
    if rc != 0:
        raise ValueError("scene has more than 64 geometries")
    return q_out, conv.astype(bool), iters, err


def collision(scene, q, targets):
    """tools.collision (tools.py:25-35) per row: q [B,15], targets [B,12] (R row-major, t)."""
    lib = load()
    f = lib.ikg_oracle_collision
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int64] + _SCENE_T + [C.c_void_p]
    f.restype = C.c_int
    a = _scene_arrays(scene)
    qq = np.ascontiguousarray(q, dtype=np.float64).reshape(-1, 15)
    tg = np.ascontiguousarray(targets, dtype=np.float64).reshape(-1, 12)
    assert len(qq) == len(tg)
    out = np.empty(len(qq), dtype=np.uint8)
    if f(qq.ctypes.data, tg.ctypes.data, len(qq), *_scene_args(a), out.ctypes.data) != 0:
        raise ValueError("scene has more than 64 geometries")
    return out.astype(bool)
