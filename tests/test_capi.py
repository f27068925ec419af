"""C-ABI surface on CPU: the library loads, exports every symbol the header
declares, validates models/arguments and reports errors through
ikg_last_error — no compute calls (there is no GPU here)."""
import ctypes as C
import os
import re

import pytest

from ikgrasp import _lib
from ikgrasp.model import load_nextage

HEADER = os.path.join(os.path.dirname(__file__), "..", "include", "ikgrasp.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?(?:int|void|char\s*\*|const char\s*\*)\s*\*?\s*(ikg_\w+)\s*\(",
                                 text, re.M)))


def test_header_declares_expected_api():
    assert declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_defaults_match_reference():
    p = _lib.default_params()
    assert p.eps == 1e-3 and p.dt == 1e-2 and p.max_iters == 1000 and p.lambda_ == 0.0
    assert _lib.load().ikg_version().startswith(b"ikgrasp")


def test_model_create_destroy():
    lib = _lib.load()
    d = _lib.model_desc(load_nextage())
    h = C.c_void_p()
    assert lib.ikg_model_create(C.byref(d), C.byref(h)) == 0 and h.value
    lib.ikg_model_destroy(h)


@pytest.mark.parametrize("mutate,msg", [
    (lambda d: setattr(d, "nq", 0), "nq"),
    (lambda d: d.axis.__setitem__(4, 7), "axis"),
    (lambda d: d.arm_q[0].__setitem__(2, 9), "arm"),
    (lambda d: d.parent.__setitem__(5, 9), "parent"),
    (lambda d: d.axis.__setitem__(12, 2), "axes differ"),
])
def test_model_create_rejects_bad_structure(mutate, msg):
    lib = _lib.load()
    d = _lib.model_desc(load_nextage())
    mutate(d)
    h = C.c_void_p()
    rc = lib.ikg_model_create(C.byref(d), C.byref(h))
    assert rc == -1
    assert msg in lib.ikg_last_error().decode()


def test_solve_rejects_bad_arguments_before_touching_the_device():
    lib = _lib.load()
    d = _lib.model_desc(load_nextage())
    h = C.c_void_p()
    assert lib.ikg_model_create(C.byref(d), C.byref(h)) == 0
    p = _lib.default_params()
    p.eps = -1.0
    rc = lib.ikg_solve_batch(h, 0, 0, None, None, 0, 4, C.byref(p), None, None, None, None, None, 0)
    assert rc == -1 and "required" in lib.ikg_last_error().decode()
    buf = (C.c_double * 64)()
    rc = lib.ikg_solve_batch(h, 0, 0, buf, buf, 0, 1, C.byref(p), buf, None, None, None, None, 0)
    assert rc == -1 and "eps" in lib.ikg_last_error().decode()
    p = _lib.default_params()
    rc = lib.ikg_solve_batch(h, 0, 5, buf, buf, 0, 1, C.byref(p), buf, None, None, None, None, 0)
    assert rc == -1 and "dtype" in lib.ikg_last_error().decode()
    rc = lib.ikg_solve_multistart(h, 0, 0, buf, 1, buf, 0, C.byref(p), buf, None, None, None, None, None, 0)
    assert rc == -1 and "S >= 1" in lib.ikg_last_error().decode()
    # launch-size limits are checked before any device work (HIP caps a grid at
    # 2^32 - 1 work items; the collision kernels run one 64-lane wave per problem)
    p.check_collision = 1
    big = (1 << 26) + 1
    rc = lib.ikg_solve_batch(h, 0, 0, buf, buf, 0, big, C.byref(p), buf, None, None, None, None, 0)
    assert rc == -1 and "too large" in lib.ikg_last_error().decode()
    rc = lib.ikg_solve_multistart(h, 0, 0, buf, 1 << 13, buf, 1 << 13, C.byref(p), buf, None, None, None, None,
                                  None, 0)
    assert rc == -1 and "too large" in lib.ikg_last_error().decode()
    p = _lib.default_params()
    p.problems_per_wave = 1
    rc = lib.ikg_solve_batch(h, 0, 0, buf, buf, 0, big, C.byref(p), buf, None, None, None, None, 0)
    assert rc == -1 and "too large" in lib.ikg_last_error().decode()
    lib.ikg_model_destroy(h)


def test_q0_shape_checks():
    import numpy as np
    from ikgrasp.solver import _q0_stride
    assert _q0_stride((15,), 8, 15) == 0
    assert _q0_stride((1, 15), 8, 15) == 0
    assert _q0_stride((8, 15), 8, 15) == 15
    for bad in ((2, 15), (8, 14), (14,), (8, 15, 1)):
        with pytest.raises(ValueError):
            _q0_stride(bad, 8, 15)


def test_no_device_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from ikgrasp.solver import IKSolver
    import numpy as np
    s = IKSolver()
    with pytest.raises(_lib.IkgError):
        s.solve(np.zeros((1, 12)), np.zeros(15))


@pytest.mark.parametrize("which", ["nextage", "tilted"])
def test_specialising_compile_runs_on_cpu(which):
    """ikg_model_specialize's hipRTC step (no GPU needed): the library's embedded
    device headers compile against a model's constant tables, both dtypes."""
    from ikgrasp.model import DualArmModel
    from ikgrasp.solver import IKSolver
    from conftest import GOLDEN
    m = load_nextage() if which == "nextage" else DualArmModel.from_urdf(
        os.path.join(GOLDEN, "tilted_dualarm.urdf"), os.path.join(GOLDEN, "tilted_cube.urdf"))
    s = IKSolver(m)
    n = C.c_size_t()
    for dtype in (_lib.IKG_F64, _lib.IKG_F32):
        rc = s.lib.ikg_debug_jit_compile(s._h, dtype, None, C.byref(n))
        assert rc == 0, s.lib.ikg_last_error().decode()
        assert n.value > 4096
    assert s.lib.ikg_model_specialize(s._h, 0, _lib.IKG_F64, 6) == -1
    assert "flags" in s.lib.ikg_last_error().decode()
    s.close()


def test_raw_launch_buffer_checks():
    """solve_into / solve_multistart_into reject buffers the kernels would
    overrun or misread, before any device call (CPU tensors fail the device check)."""
    import torch
    from ikgrasp.solver import IKSolver
    s = IKSolver()
    B = 4
    tg = torch.zeros((B, 12), dtype=torch.float64)
    good = dict(q_out=torch.zeros((B, 15), dtype=torch.float64), conv=torch.zeros(B, dtype=torch.uint8),
                iters=torch.zeros(B, dtype=torch.int32), err=torch.zeros((B, 2), dtype=torch.float64))
    with pytest.raises(ValueError, match="device tensor"):  # CPU tensors, shapes right
        s.solve_into(tg, torch.zeros(15, dtype=torch.float64), *good.values(), _lib.IKG_F64, 0)
    bad = dict(good, q_out=torch.zeros((B, 14), dtype=torch.float64))
    with pytest.raises(ValueError, match="q_out"):
        s._check_out(B, _lib.IKG_F64, tg, *bad.values())
    bad = dict(good, iters=torch.zeros(B, dtype=torch.int64))
    with pytest.raises(ValueError, match="iters"):
        s._check_out(B, _lib.IKG_F64, tg, *bad.values())
    with pytest.raises(ValueError, match="q_out"):  # fp32 launch code, fp64 buffers
        s._check_out(B, _lib.IKG_F32, tg.float(), *good.values())
    s.close()


def test_specialising_compile_cache(tmp_path, monkeypatch):
    """IKG_JIT_CACHE_DIR: the first compile writes the code object, a second
    model with the same tables loads it without compiling (and gets the same bytes)."""
    import time
    from ikgrasp.solver import IKSolver
    monkeypatch.setenv("IKG_JIT_CACHE_DIR", str(tmp_path))
    n = C.c_size_t()
    a = IKSolver()
    assert a.lib.ikg_debug_jit_compile(a._h, _lib.IKG_F32, str(tmp_path / "a.co").encode(), C.byref(n)) == 0
    files = sorted(p.name for p in tmp_path.glob("ikg_jit_*.co"))
    assert len(files) == 1
    b = IKSolver()
    t0 = time.perf_counter()
    assert b.lib.ikg_debug_jit_compile(b._h, _lib.IKG_F32, str(tmp_path / "b.co").encode(), C.byref(n)) == 0
    assert time.perf_counter() - t0 < 0.5  # a hipRTC compile takes ~1.5 s here
    assert (tmp_path / "a.co").read_bytes() == (tmp_path / "b.co").read_bytes()
    a.close()
    b.close()


def test_specialising_compile_cache_ignores_damaged_files(tmp_path, monkeypatch):
    """A cache file that is not an ELF code object is recompiled and replaced."""
    from ikgrasp.solver import IKSolver
    monkeypatch.setenv("IKG_JIT_CACHE_DIR", str(tmp_path))
    n = C.c_size_t()
    a = IKSolver()
    assert a.lib.ikg_debug_jit_compile(a._h, _lib.IKG_F32, None, C.byref(n)) == 0
    (f,) = list(tmp_path.glob("ikg_jit_*.co"))
    good = f.read_bytes()
    f.write_bytes(b"not a code object")
    b = IKSolver()
    assert b.lib.ikg_debug_jit_compile(b._h, _lib.IKG_F32, None, C.byref(n)) == 0
    assert n.value == len(good) and f.read_bytes() == good
    a.close()
    b.close()
