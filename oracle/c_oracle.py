"""ctypes loader for the C oracle (oracle/ikg_oracle.c) — test/baseline
infrastructure only (tests/, smoke(), bench.py cpu_baseline)."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libikg_oracle.so")
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
