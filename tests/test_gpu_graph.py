"""HIP graph capture of the C-ABI launches (torch.cuda.CUDAGraph on ROCm is a
hipGraph): a solve captured once and replayed must give the same outputs as
direct launches.  Covers the batch solve (one kernel), the multi-start solve
(stream-ordered workspace allocation inside the capture) and the solve with
the collision term (pre-screen, compaction, memsets, continuation)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bufs(torch, B, dt, dev, nq=15):
    return (torch.empty((B, nq), dtype=dt, device=dev), torch.empty(B, dtype=torch.uint8, device=dev),
            torch.empty(B, dtype=torch.int32, device=dev), torch.empty((B, 2), dtype=dt, device=dev))


def _same(a, b):
    return all(bool(torch_equal(x, y)) for x, y in zip(a, b))



def torch_equal(x, y):
    import torch
    return torch.equal(x, y)


@pytest.mark.parametrize("collision", [False, True])
def test_batch_solve_replays_from_a_graph(collision):
    import torch
    from ikgrasp import _lib
    from ikgrasp.collision import load_nextage_scene
    from ikgrasp.solver import IKSolver
    from ikgrasp.workload import uniform_targets
    dev = torch.device("cuda", 0)
    s = IKSolver(device=0, scene=load_nextage_scene() if collision else None)
    tg = torch.tensor(uniform_targets(1024, seed=3), dtype=torch.float64, device=dev)
    q0 = torch.zeros(15, dtype=torch.float64, device=dev)
    ref = _bufs(torch, 1024, torch.float64, dev)
    s.solve_into(tg, q0, *ref, _lib.IKG_F64, torch.cuda.current_stream().cuda_stream, check_collision=collision)
    torch.cuda.synchronize()
    out = _bufs(torch, 1024, torch.float64, dev)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm up off the default stream, as torch recommends before capture
        s.solve_into(tg, q0, *out, _lib.IKG_F64, side.cuda_stream, check_collision=collision)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    for x in out:
        x.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s.solve_into(tg, q0, *out, _lib.IKG_F64, torch.cuda.current_stream().cuda_stream,
                     check_collision=collision)
    for x in out:
        x.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert _same(out, ref), _diff(out, ref)
    # replays read the inputs in place: new targets, new answers
    tg.copy_(torch.tensor(uniform_targets(1024, seed=4), dtype=torch.float64, device=dev))
    g.replay()
    torch.cuda.synchronize()
    ref2 = _bufs(torch, 1024, torch.float64, dev)
    s.solve_into(tg, q0, *ref2, _lib.IKG_F64, torch.cuda.current_stream().cuda_stream, check_collision=collision)
    torch.cuda.synchronize()
    assert _same(out, ref2), _diff(out, ref2)
    s.close()


def test_multistart_replays_from_a_graph():
    import torch
    from ikgrasp import _lib
    from ikgrasp.solver import IKSolver
    from ikgrasp.workload import random_seeds, uniform_targets
    dev = torch.device("cuda", 0)
    s = IKSolver(device=0)
    T, S = 64, 16
    tg = torch.tensor(uniform_targets(T, seed=5), dtype=torch.float32, device=dev)
    seeds = torch.tensor(random_seeds(s.model, S, seed=6), dtype=torch.float32, device=dev)
    ref = _bufs(torch, T, torch.float32, dev) + (torch.empty(T, dtype=torch.int32, device=dev),)
    s.solve_multistart_into(tg, seeds, *ref, _lib.IKG_F32, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = _bufs(torch, T, torch.float32, dev) + (torch.empty(T, dtype=torch.int32, device=dev),)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        s.solve_multistart_into(tg, seeds, *out, _lib.IKG_F32, side.cuda_stream)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s.solve_multistart_into(tg, seeds, *out, _lib.IKG_F32, torch.cuda.current_stream().cuda_stream)
    for x in out:
        x.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert _same(out, ref)
    s.close()


def _diff(out, ref):
    return [(i, float((x.double() - y.double()).abs().max())) for i, (x, y) in enumerate(zip(out, ref))
            if not torch_equal(x, y)]


def test_specialised_kernels_replay_from_a_graph():
    """The hipRTC module launch (hipModuleLaunchKernel) is captured too."""
    import os

    import torch
    from conftest import GOLDEN
    from ikgrasp import _lib
    from ikgrasp.model import DualArmModel
    from ikgrasp.solver import IKSolver
    dev = torch.device("cuda", 0)
    m = DualArmModel.from_urdf(os.path.join(GOLDEN, "tilted_dualarm.urdf"), os.path.join(GOLDEN, "tilted_cube.urdf"))
    s = IKSolver(m, device=0, specialize=True)
    gc = np.load(os.path.join(GOLDEN, "generic_cases.npz"))
    tg = torch.tensor(gc["targets"], dtype=torch.float64, device=dev)
    q0 = torch.tensor(gc["q0"], dtype=torch.float64, device=dev)
    B, nq = tg.shape[0], s.nq  # the tilted robot has 14 joints
    ref = _bufs(torch, B, torch.float64, dev, nq)
    s.solve_into(tg, q0, *ref, _lib.IKG_F64, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert s.is_specialized("f64")
    out = _bufs(torch, B, torch.float64, dev, nq)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s.solve_into(tg, q0, *out, _lib.IKG_F64, torch.cuda.current_stream().cuda_stream)
    for x in out:
        x.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    assert _same(out, ref), _diff(out, ref)
    s.close()
