"""Scratch memory of the C-ABI (include/ikgrasp.h "Scratch memory", "Graphs";
csrc/ikg_launch.hpp ws_*).

* An uncaptured solve's scratch (the collision records are the large item:
  656 MB at C2 fp64) comes from a stream-ordered pool the model owns, which
  keeps it reserved for the next solve.  ikg_model_trim releases it without
  destroying the model, ikg_model_destroy destroys the pool.  A first model
  solved and destroyed beforehand absorbs what the HIP runtime itself keeps
  after a first launch of these kernels (code objects, the private-segment
  allocation of kernels that use scratch, memory it keeps mapped to back
  pools), which is not the model's.
* A captured solve's scratch belongs to its graph; once the graph is
  destroyed a later capture on the same model reuses it, so a workload that
  recaptures every cycle and never solves uncaptured holds a bounded number
  of buffers."""
import ctypes as C
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_bytes():
    import torch
    torch.cuda.synchronize()
    return torch.cuda.mem_get_info(0)[0]


def _pool(s):
    """(reserved, used) bytes of the solver's model's scratch pools."""
    from ikgrasp import _lib
    lib = _lib.load()
    lib.ikg_debug_ws_pool.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    r, u = C.c_int64(), C.c_int64()
    assert lib.ikg_debug_ws_pool(s._h, C.byref(r), C.byref(u)) == 0
    return r.value, u.value


def test_pool_scratch_is_reused_and_released():
    """A C2 collision solve's scratch (656 MB of fp64 records) comes from the
    model's pool.  What the device's free-memory figure can show: a first
    model, solved and destroyed, leaves memory the HIP runtime keeps mapped
    (its pools' released memory, the private segments of the kernels that use
    scratch); a second model then solves, repeats, trims and solves again
    without taking any more of the device, and after ikg_model_destroy the
    figure is where it was before the second model existed -- nothing the
    model allocated stays with it.  ikg_model_trim and repeated solves keep the
    answers bit for bit.  The pool's own reservation counters are printed
    (hipMemPoolAttrReservedMemCurrent; this runtime reports 0 for them, so
    they are not gated)."""
    from ikgrasp.collision import load_nextage_scene
    from ikgrasp.solver import IKSolver
    from ikgrasp.workload import uniform_targets
    tg = uniform_targets(4096, seed=0)
    scene = load_nextage_scene()
    free_start = _free_bytes()
    warm = IKSolver(device=0, scene=scene)
    ref = warm.solve(tg, np.zeros(15), check_collision=True)
    warm.close()
    free0 = _free_bytes()
    s = IKSolver(device=0, scene=scene)
    a = s.solve(tg, np.zeros(15), check_collision=True)
    free1 = _free_bytes()
    b = s.solve(tg, np.zeros(15), check_collision=True)
    r1, u1 = _pool(s)
    s.trim()
    c = s.solve(tg, np.zeros(15), check_collision=True)
    free2 = _free_bytes()
    for x in (a, b, c):
        assert np.array_equal(x.q, ref.q) and np.array_equal(x.iters, ref.iters)
    s.close()
    free3 = _free_bytes()
    print(f"device free memory (GB): {free_start / 1e9:.3f} at start, {free0 / 1e9:.3f} after a first model "
          f"(solved, destroyed), {free1 / 1e9:.3f} after a second model's solve, {free2 / 1e9:.3f} after its trim "
          f"and another solve, {free3 / 1e9:.3f} after ikg_model_destroy; pool counters reserved {r1}, used {u1}")
    assert free0 - free1 < 64e6 and free0 - free2 < 64e6  # the runtime's memory serves the second model
    assert free0 - free3 < 64e6                            # nothing stays with the destroyed model


def test_recapture_without_uncaptured_solves_stays_bounded():
    """Capture a collision solve into a new graph every cycle, replay it,
    destroy the previous cycle's graph, never solve uncaptured: the buffers
    held (live + pending) stay within two cycles' worth (a destroyed graph's
    release may lag its destroy by one cycle), and every replay equals a
    direct solve."""
    import torch
    from ikgrasp import _lib
    from ikgrasp.collision import load_nextage_scene
    from ikgrasp.solver import IKSolver
    from ikgrasp.workload import uniform_targets
    lib = _lib.load()
    lib.ikg_debug_ws_count.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]

    def counts(s):
        live, pend = C.c_int64(), C.c_int64()
        assert lib.ikg_debug_ws_count(s._h, C.byref(live), C.byref(pend)) == 0
        return live.value, pend.value

    dev = torch.device("cuda", 0)
    s = IKSolver(device=0, scene=load_nextage_scene())
    B = 512
    tg = torch.tensor(uniform_targets(B, seed=9), dtype=torch.float64, device=dev)
    q0 = torch.zeros(15, dtype=torch.float64, device=dev)

    def bufs():
        return (torch.empty((B, 15), dtype=torch.float64, device=dev), torch.empty(B, dtype=torch.uint8, device=dev),
                torch.empty(B, dtype=torch.int32, device=dev), torch.empty((B, 2), dtype=torch.float64, device=dev))

    ref = bufs()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up off the default stream (the only uncaptured solve)
        s.solve_into(tg, q0, *ref, _lib.IKG_F64, side.cuda_stream, check_collision=True)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    assert counts(s) == (0, 0)
    out = bufs()
    prev, per_cycle, seen = None, None, []
    for k in range(8):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            s.solve_into(tg, q0, *out, _lib.IKG_F64, torch.cuda.current_stream().cuda_stream,
                         check_collision=True)
        for x in out:
            x.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert all(torch.equal(x, y) for x, y in zip(out, ref)), k
        if per_cycle is None:
            per_cycle = counts(s)[0]
            assert per_cycle >= 1
        if prev is not None:
            prev.reset()  # destroys the previous cycle's graph and its executable
        prev = g
        time.sleep(0.01)
        live, pend = counts(s)
        seen.append((live, pend))
        assert live + pend <= 3 * per_cycle, (k, seen)
    print(f"buffers per captured solve {per_cycle}; (live, pending) per cycle {seen}")
    prev.reset()
    s.trim()  # frees what is pending
    for _ in range(100):
        if counts(s)[1] == 0:
            break
        time.sleep(0.02)
        s.trim()
    assert counts(s) == (0, 0)
    s.close()
