"""Batched solver front-end over the C-ABI.

`IKSolver` accepts either numpy arrays (host memory: the library stages them
through device scratch) or torch tensors already resident on a ROCm device
(device pointers, launched on torch's current stream — the zero-copy path the
benchmark uses).  The HIP kernel is the only compute path.
"""
from __future__ import annotations

import ctypes as C
import warnings
from dataclasses import dataclass

import numpy as np

from . import _lib
from .model import DualArmModel, load_nextage

_DT = {"f64": (_lib.IKG_F64, np.float64), "f32": (_lib.IKG_F32, np.float32)}


def _dtype(dtype):
    if dtype in ("f64", "float64", np.float64, "double"):
        return _DT["f64"]
    if dtype in ("f32", "float32", np.float32, "float"):
        return _DT["f32"]
    try:
        import torch
        if dtype == torch.float64:
            return _DT["f64"]
        if dtype == torch.float32:
            return _DT["f32"]
    except ImportError:  # pragma: no cover
        pass
    raise ValueError(f"unsupported dtype {dtype!r}")


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _q0_stride(shape, B: int, nq: int) -> int:
    """Row stride of a q0 array for ikg_solve_batch: [nq] or [1, nq] broadcast
    (stride 0), [B, nq] one row per target (stride nq).  Anything else would
    make the kernel read past the end of q0, so it is rejected here."""
    shape = tuple(shape)
    if shape == (nq,) or shape == (1, nq):
        return 0
    if shape == (B, nq):
        return nq
    raise ValueError(f"q0 must be [{nq}], [1,{nq}] or [{B},{nq}], got {list(shape)}")


@dataclass
class Solution:
    q: object            # [B, nq]
    converged: object    # [B] bool/uint8
    iters: object        # [B] int32
    err: object          # [B, 2] |log6| left/right at q
    best_seed: object = None


class IKSolver:
    """Owns one native model (`ikg_model_create`)."""

    def __init__(self, model: DualArmModel | None = None, device: int = 0, scene=None, specialize="auto"):
        """`scene`: an ikgrasp.collision.CollisionScene to attach (see set_collision).
        `specialize`: "auto" compiles model-specialised pair kernels
        (ikg_model_specialize) on a model's first solve per dtype and device
        unless the prebuilt library already has its specialisation (Nextage
        class); a failed compile warns and keeps the prebuilt generic kernel.
        True: always specialise, raising on failure.  False: prebuilt only."""
        if specialize not in ("auto", True, False):
            raise ValueError(f"specialize must be 'auto', True or False, got {specialize!r}")
        self._specialize = specialize
        self._specialized = set()
        self.lib = _lib.load()
        self.model = model if model is not None else load_nextage()
        self.desc = _lib.model_desc(self.model)
        h = C.c_void_p()
        _lib.check(self.lib.ikg_model_create(C.byref(self.desc), C.byref(h)))
        self._h = h
        self.device = device
        self.scene = None
        if scene is not None:
            self.set_collision(scene)

    def set_collision(self, scene):
        """Attach the collision scene (ikg_model_set_collision); enables
        `check_collision=True` solves and `collision()` queries."""
        self._cdesc = _lib.collision_desc(scene)
        _lib.check(self.lib.ikg_model_set_collision(self._h, C.byref(self._cdesc)))
        self.scene = scene

    def _auto_specialize(self, device, code):
        if self._specialize is False or (device, code) in self._specialized:
            return
        self._specialized.add((device, code))
        flags = _lib.IKG_SPECIALIZE_IF_GENERIC if self._specialize == "auto" else 0
        rc = self.lib.ikg_model_specialize(self._h, device, code, flags)
        if rc != 0:
            msg = self.lib.ikg_last_error().decode()
            if self._specialize is True:
                raise _lib.IkgError(rc, msg)
            warnings.warn(f"model specialisation failed, using the prebuilt generic kernels: {msg}")

    def _native_solve(self, h, device, code, *rest):
        self._auto_specialize(device, code)
        return self.lib.ikg_solve_batch(h, device, code, *rest)

    def _native_multistart(self, h, device, code, *rest):
        self._auto_specialize(device, code)
        return self.lib.ikg_solve_multistart(h, device, code, *rest)

    def specialize(self, dtype="f64", device=None):
        """Compile the pair-layout kernels against this model's tables
        (ikg_model_specialize, hipRTC) for `dtype` on `device` (default: the
        solver's); later solves there use them.  Seconds for the first device."""
        code, _ = _dtype(dtype)
        _lib.check(self.lib.ikg_model_specialize(self._h, self.device if device is None else device, code, 0))

    def is_specialized(self, dtype="f64", device=None) -> bool:
        code, _ = _dtype(dtype)
        return bool(self.lib.ikg_model_is_specialized(self._h, self.device if device is None else device, code))

    def trim(self):
        """Give the scratch memory this model's pools keep for later solves
        back to the driver (ikg_model_trim); the solver stays usable."""
        _lib.check(self.lib.ikg_model_trim(self._h))

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.ikg_model_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    @property
    def nq(self) -> int:
        return self.model.nq

    def params(self, eps=1e-3, dt=1e-2, max_iters=1000, lam=0.0, variant=_lib.IKG_VARIANT_AUTO, ppw=0,
               check_collision=False):
        """check_collision: reference `success` (converged AND collision-free,
        iterating on while converged-but-colliding, inverse_geometry.py:70)."""
        return _lib.default_params(eps=eps, dt=dt, max_iters=max_iters, lambda_=lam, variant=variant,
                                   problems_per_wave=ppw, check_collision=int(bool(check_collision)))

    # ------------------------------------------------------------------ batch
    def solve(self, targets, q0, dtype="f64", stream=None, **kw) -> Solution:
        """targets [B,12] cube placements; q0 [nq] (broadcast) or [B,nq]."""
        prm = self.params(**kw)
        if _is_torch(targets):
            return self._solve_torch(targets, q0, prm, stream)
        code, npt = _dtype(dtype)
        tg = np.ascontiguousarray(targets, dtype=npt).reshape(-1, 12)
        B = tg.shape[0]
        q = np.ascontiguousarray(q0, dtype=npt)
        stride = _q0_stride(q.shape, B, self.nq)
        q_out = np.empty((B, self.nq), dtype=npt)
        conv = np.empty(B, dtype=np.uint8)
        iters = np.empty(B, dtype=np.int32)
        err = np.empty((B, 2), dtype=npt)
        _lib.check(self._native_solve(
            self._h, self.device, code, tg.ctypes.data, q.ctypes.data, stride, B, C.byref(prm),
            q_out.ctypes.data, conv.ctypes.data, iters.ctypes.data, err.ctypes.data, None,
            _lib.IKG_FLAG_HOST_POINTERS))
        return Solution(q_out, conv.astype(bool), iters, err)

    def _solve_torch(self, targets, q0, prm, stream):
        import torch
        code, _ = _dtype(targets.dtype)
        if not targets.is_cuda:
            raise ValueError("torch targets must live on a ROCm device (or pass numpy arrays)")
        dev = targets.device
        tg = targets.contiguous().view(-1, 12)
        B = tg.shape[0]
        q = q0.to(device=dev, dtype=targets.dtype).contiguous()
        stride = _q0_stride(q.shape, B, self.nq)
        q_out = torch.empty((B, self.nq), dtype=targets.dtype, device=dev)
        conv = torch.empty(B, dtype=torch.uint8, device=dev)
        iters = torch.empty(B, dtype=torch.int32, device=dev)
        err = torch.empty((B, 2), dtype=targets.dtype, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        _lib.check(self._native_solve(
            self._h, dev.index or 0, code, tg.data_ptr(), q.data_ptr(), stride, B, C.byref(prm),
            q_out.data_ptr(), conv.data_ptr(), iters.data_ptr(), err.data_ptr(), C.c_void_p(s), 0))
        return Solution(q_out, conv.bool(), iters, err)

    def _check_out(self, B, dtype_code, targets, q_out, conv, iters, err, best=None):
        """Preallocated torch buffers of the raw launches: shapes, dtypes and
        contiguity the kernels assume (a q_out narrower than nq would be
        written past its end)."""
        import torch
        fdt = torch.float64 if dtype_code == _lib.IKG_F64 else torch.float32
        want = [(targets, (B, 12), fdt, "targets"), (q_out, (B, self.nq), fdt, "q_out"),
                (conv, (B,), torch.uint8, "converged"), (iters, (B,), torch.int32, "iters"),
                (err, (B, 2), fdt, "err")]
        if best is not None:
            want.append((best, (B,), torch.int32, "best_seed"))
        for t, shape, dt, name in want:
            if tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous {dt} tensor of shape {list(shape)}, got "
                                 f"{t.dtype} {list(t.shape)}")
        for t, _, _, name in want:
            if not t.is_cuda:
                raise ValueError(f"{name} must be a device tensor")

    def solve_into(self, targets, q0, q_out, conv, iters, err, dtype_code, stream_handle, **kw):
        """Raw device-pointer launch (all tensors preallocated; used by bench.py)."""
        prm = self.params(**kw)
        self._check_out(targets.shape[0], dtype_code, targets, q_out, conv, iters, err)
        if not q0.is_contiguous() or q0.dtype != targets.dtype:
            raise ValueError("q0 must be contiguous and of the targets' dtype")
        stride = _q0_stride(q0.shape, targets.shape[0], self.nq)
        _lib.check(self._native_solve(
            self._h, targets.device.index or 0, dtype_code, targets.data_ptr(), q0.data_ptr(), stride,
            targets.shape[0], C.byref(prm), q_out.data_ptr(), conv.data_ptr(), iters.data_ptr(),
            err.data_ptr(), C.c_void_p(stream_handle), 0))

    def solve_multistart_into(self, targets, seeds, q_out, conv, iters, err, best, dtype_code, stream_handle, **kw):
        """Raw device-pointer multi-start launch (preallocated torch tensors; bench.py)."""
        prm = self.params(**kw)
        if seeds.dim() != 2 or seeds.shape[1] != self.nq:
            raise ValueError(f"seeds must be [S,{self.nq}], got {list(seeds.shape)}")
        if not seeds.is_contiguous() or seeds.dtype != targets.dtype:
            raise ValueError("seeds must be contiguous and of the targets' dtype")
        self._check_out(targets.shape[0], dtype_code, targets, q_out, conv, iters, err, best)
        _lib.check(self._native_multistart(
            self._h, targets.device.index or 0, dtype_code, targets.data_ptr(), targets.shape[0], seeds.data_ptr(),
            seeds.shape[0], C.byref(prm), q_out.data_ptr(), conv.data_ptr(), iters.data_ptr(), err.data_ptr(),
            best.data_ptr(), C.c_void_p(stream_handle), 0))

    # ------------------------------------------------------------------ multistart
    def solve_multistart(self, targets, seeds, dtype="f64", **kw) -> Solution:
        """S seeds x T targets -> best seed per target (ikg_solve_multistart)."""
        prm = self.params(**kw)
        code, npt = _dtype(dtype)
        tg = np.ascontiguousarray(targets, dtype=npt).reshape(-1, 12)
        sd = np.ascontiguousarray(seeds, dtype=npt).reshape(-1, self.nq)
        T, S = tg.shape[0], sd.shape[0]
        q_out = np.empty((T, self.nq), dtype=npt)
        conv = np.empty(T, dtype=np.uint8)
        iters = np.empty(T, dtype=np.int32)
        err = np.empty((T, 2), dtype=npt)
        best = np.empty(T, dtype=np.int32)
        _lib.check(self._native_multistart(
            self._h, self.device, code, tg.ctypes.data, T, sd.ctypes.data, S, C.byref(prm),
            q_out.ctypes.data, conv.ctypes.data, iters.ctypes.data, err.ctypes.data, best.ctypes.data, None,
            _lib.IKG_FLAG_HOST_POINTERS))
        return Solution(q_out, conv.astype(bool), iters, err, best)

    # ------------------------------------------------------------------ collision
    def collision(self, q, targets, dtype="f64"):
        """tools.collision(robot, q) with the cube at each target: q [B,nq],
        targets [B,12] -> bool [B] (numpy) or uint8 tensor (torch, device)."""
        if _is_torch(q):
            import torch
            code, _ = _dtype(q.dtype)
            qq = q.contiguous().view(-1, self.nq)
            tg = targets.to(device=q.device, dtype=q.dtype).contiguous().view(-1, 12)
            out = torch.empty(qq.shape[0], dtype=torch.uint8, device=q.device)
            s = torch.cuda.current_stream(q.device).cuda_stream
            _lib.check(self.lib.ikg_collision_batch(self._h, q.device.index or 0, code, qq.data_ptr(), tg.data_ptr(),
                                                    qq.shape[0], out.data_ptr(), C.c_void_p(s), 0))
            return out
        code, npt = _dtype(dtype)
        qq = np.ascontiguousarray(q, dtype=npt).reshape(-1, self.nq)
        tg = np.ascontiguousarray(np.broadcast_to(np.asarray(targets, dtype=npt).reshape(-1, 12), (qq.shape[0], 12)))
        out = np.empty(qq.shape[0], dtype=np.uint8)
        _lib.check(self.lib.ikg_collision_batch(self._h, self.device, code, qq.ctypes.data, tg.ctypes.data,
                                                qq.shape[0], out.ctypes.data, None, _lib.IKG_FLAG_HOST_POINTERS))
        return out.astype(bool)

    # ------------------------------------------------------------------ planner queries
    def distance(self, q, targets, pair_idx, dtype="f64") -> np.ndarray:
        """min over the listed active pairs of the pair distance (hpp-fcl
        computeDistance().min_distance; <= 0 when intersecting) for each
        configuration: q [B,nq], targets [B,12] (or one row, broadcast) -> [B]."""
        code, npt = _dtype(dtype)
        qq = np.ascontiguousarray(q, dtype=npt).reshape(-1, self.nq)
        tg = np.ascontiguousarray(np.broadcast_to(np.asarray(targets, dtype=npt).reshape(-1, 12), (qq.shape[0], 12)))
        idx = np.ascontiguousarray(pair_idx, dtype=np.int32).reshape(-1)
        out = np.empty(qq.shape[0], dtype=npt)
        _lib.check(self.lib.ikg_distance_batch(self._h, self.device, code, qq.ctypes.data, tg.ctypes.data,
                                               qq.shape[0], idx.ctypes.data, idx.size, out.ctypes.data, None,
                                               _lib.IKG_FLAG_HOST_POINTERS))
        return out

    def pair_distances(self, q, targets, pair_idx, dtype="f64") -> np.ndarray:
        """Each listed pair's distance: [B, len(pair_idx)] (one query per pair)."""
        return np.stack([self.distance(q, targets, [k], dtype) for k in pair_idx], axis=1)

    def target_env(self, targets, geoms, dtype="f64") -> np.ndarray:
        """The scene's target geometry at each placement [B,12] against the
        listed world-fixed geometries -> bool [B] (path.py:51-52)."""
        code, npt = _dtype(dtype)
        tg = np.ascontiguousarray(targets, dtype=npt).reshape(-1, 12)
        g = np.ascontiguousarray(geoms, dtype=np.int32).reshape(-1)
        out = np.empty(tg.shape[0], dtype=np.uint8)
        _lib.check(self.lib.ikg_target_env_batch(self._h, self.device, code, tg.ctypes.data, tg.shape[0],
                                                 g.ctypes.data, g.size, out.ctypes.data, None,
                                                 _lib.IKG_FLAG_HOST_POINTERS))
        return out.astype(bool)

    # ------------------------------------------------------------------ log6
    def log6(self, M, dtype="f64") -> np.ndarray:
        """pin.log6 of placements [B,12] -> [B,6] ([v; w])."""
        code, npt = _dtype(dtype)
        mm = np.ascontiguousarray(M, dtype=npt).reshape(-1, 12)
        out = np.empty((mm.shape[0], 6), dtype=npt)
        _lib.check(self.lib.ikg_log6_batch(self.device, code, mm.ctypes.data, mm.shape[0], out.ctypes.data, None,
                                           _lib.IKG_FLAG_HOST_POINTERS))
        return out

    # ------------------------------------------------------------------ FK
    def fk(self, q, dtype="f64") -> np.ndarray:
        """Hands placements [B, 2, 12] (R row-major, t) for q [B, nq]."""
        code, npt = _dtype(dtype)
        qq = np.ascontiguousarray(q, dtype=npt).reshape(-1, self.nq)
        out = np.empty((qq.shape[0], 2, 12), dtype=npt)
        _lib.check(self.lib.ikg_fk_batch(self._h, self.device, code, qq.ctypes.data, qq.shape[0],
                                         out.ctypes.data, None, _lib.IKG_FLAG_HOST_POINTERS))
        return out

    # ------------------------------------------------------------------ controller kinematics
    FRAME_KIN_OUTPUTS = ("placement", "velocity", "J", "dJ", "dJv", "err", "derr")

    def frame_kinematics(self, q, v=None, q_des=None, v_des=None, rf=_lib.IKG_LOCAL_WORLD_ALIGNED,
                         outputs=("placement", "velocity", "J", "dJ", "dJv"), dtype="f64", stream=None) -> dict:
        """ikg_frame_kinematics_batch: per state and hand (LARM_EFF, RARM_EFF)
        the kinematic terms of control.py:284-345 in reference frame `rf`.
        q, v [B,nq] (numpy, or torch tensors on a ROCm device); q_des / v_des
        only for 'err' / 'derr'.  Returns {name: array} with placement [B,2,12],
        velocity [B,2,6], J / dJ [B,12,nq], dJv / err / derr [B,12]."""
        unknown = set(outputs) - set(self.FRAME_KIN_OUTPUTS)
        if unknown:
            raise ValueError(f"unknown outputs {sorted(unknown)}")
        nq = self.nq
        shapes = {"placement": (2, 12), "velocity": (2, 6), "J": (12, nq), "dJ": (12, nq), "dJv": (12,),
                  "err": (12,), "derr": (12,)}
        if ("err" in outputs or "derr" in outputs) and q_des is None:
            raise ValueError("err/derr need q_des")
        if _is_torch(q):
            import torch
            code, _ = _dtype(q.dtype)
            dev = q.device
            prep = lambda x: None if x is None else x.to(device=dev, dtype=q.dtype).contiguous().view(-1, nq)
            qq, vv, qd, vd = prep(q), prep(v), prep(q_des), prep(v_des)
            B = qq.shape[0]
            for name, x in (("v", vv), ("q_des", qd), ("v_des", vd)):
                if x is not None and x.shape[0] != B:
                    raise ValueError(f"{name} has {x.shape[0]} rows, q has {B}")
            res = {k: torch.empty((B,) + shapes[k], dtype=q.dtype, device=dev) for k in outputs}
            ptr = lambda x: None if x is None else x.data_ptr()
            out = _lib.FrameKinOut(*[ptr(res.get(k)) for k in self.FRAME_KIN_OUTPUTS])
            s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
            _lib.check(self.lib.ikg_frame_kinematics_batch(
                self._h, dev.index or 0, code, ptr(qq), ptr(vv), ptr(qd), ptr(vd), B, int(rf), C.byref(out),
                C.c_void_p(s), 0))
            return res
        code, npt = _dtype(dtype)
        prep = lambda x: None if x is None else np.ascontiguousarray(x, dtype=npt).reshape(-1, nq)
        qq, vv, qd, vd = prep(q), prep(v), prep(q_des), prep(v_des)
        B = qq.shape[0]
        for name, x in (("v", vv), ("q_des", qd), ("v_des", vd)):
            if x is not None and x.shape[0] != B:
                raise ValueError(f"{name} has {x.shape[0]} rows, q has {B}")
        res = {k: np.empty((B,) + shapes[k], dtype=npt) for k in outputs}
        ptr = lambda x: None if x is None else x.ctypes.data
        out = _lib.FrameKinOut(*[ptr(res.get(k)) for k in self.FRAME_KIN_OUTPUTS])
        _lib.check(self.lib.ikg_frame_kinematics_batch(
            self._h, self.device, code, ptr(qq), ptr(vv), ptr(qd), ptr(vd), B, int(rf), C.byref(out), None,
            _lib.IKG_FLAG_HOST_POINTERS))
        return res
