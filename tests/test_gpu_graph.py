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
    assert _same(out, ref2), _diff(out, ref2) + _rows(out, ref2, ref)
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


def _rows(out, ref, prev):
    """Which problems differ, and whether the replay's q is another solve's:
    the previous targets' answer at the same index, or some other row."""
    q, c, it, e = (x.cpu().numpy() for x in out)
    q2, c2, it2, e2 = (x.cpu().numpy() for x in ref)
    qp = prev[0].cpu().numpy()
    bad = np.nonzero(np.abs(q - q2).max(axis=1) > 0)[0]
    rows = []
    for i in bad[:8]:
        same_prev = bool(np.array_equal(q[i], qp[i]))
        other = np.nonzero((np.abs(q2 - q[i]).max(axis=1) == 0))[0].tolist()[:3]
        rows.append(dict(i=int(i), conv=(int(c[i]), int(c2[i])), iters=(int(it[i]), int(it2[i])),
                         dq=float(np.abs(q[i] - q2[i]).max()), joint=int(np.abs(q[i] - q2[i]).argmax()),
                         err=(e[i].tolist(), e2[i].tolist()), equals_previous_answer=same_prev,
                         equals_rows_of_direct=other))
    return [f"{len(bad)} rows differ"] + rows


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


@pytest.mark.skipif(not __import__("os").environ.get("IKG_GRAPH_DIAG"), reason="diagnostic (IKG_GRAPH_DIAG=1)")
def test_diag_collision_replays():
    """Diagnostic: one captured solve with the collision term replayed on six
    target sets, each compared with a direct solve; every differing row is
    printed with its first passing iterate k0 (solve without the term)."""
    import torch
    from ikgrasp import _lib
    from ikgrasp.collision import load_nextage_scene
    from ikgrasp.solver import IKSolver
    from ikgrasp.workload import uniform_targets
    dev = torch.device("cuda", 0)
    s = IKSolver(device=0, scene=load_nextage_scene())
    sh = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    tg = torch.tensor(uniform_targets(1024, seed=3), dtype=torch.float64, device=dev)
    q0 = torch.zeros(15, dtype=torch.float64, device=dev)
    out = _bufs(torch, 1024, torch.float64, dev)
    s.solve_into(tg, q0, *out, _lib.IKG_F64, sh(), check_collision=True)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s.solve_into(tg, q0, *out, _lib.IKG_F64, sh(), check_collision=True)
    bad_total = 0
    for seed in range(3, 9):
        tg.copy_(torch.tensor(uniform_targets(1024, seed=seed), dtype=torch.float64, device=dev))
        g.replay()
        torch.cuda.synchronize()
        ref = _bufs(torch, 1024, torch.float64, dev)
        s.solve_into(tg, q0, *ref, _lib.IKG_F64, sh(), check_collision=True)
        free = _bufs(torch, 1024, torch.float64, dev)
        s.solve_into(tg, q0, *free, _lib.IKG_F64, sh(), check_collision=False)
        torch.cuda.synchronize()
        q, c, it, e = (x.cpu().numpy() for x in out)
        q2, c2, it2, e2 = (x.cpu().numpy() for x in ref)
        k0 = free[2].cpu().numpy()
        bad = np.nonzero((np.abs(q - q2).max(axis=1) > 0) | (c != c2) | (it != it2))[0]
        bad_total += len(bad)
        print(f"\n[diag] replay on seed {seed}: {len(bad)} rows differ; ran on (k0<1000, failed): "
              f"{int(((k0 < 1000) & (c2 == 0)).sum())}")
        for i in bad[:6]:
            print(f"[diag]   row {i}: k0={k0[i]} conv {c[i]}/{c2[i]} iters {it[i]}/{it2[i]} "
                  f"q_replay={np.round(q[i], 4).tolist()} q_direct={np.round(q2[i], 4).tolist()} "
                  f"err {e[i].tolist()} / {e2[i].tolist()}")
    s.close()
    assert bad_total == 0


def test_captured_scratch_lives_with_its_graph():
    """a captured solve's scratch (records, workspaces) belongs to
    the graph (a hipGraph user object), not to the model: it is held while the
    graph lives, and freed on the model's next solve once the graph is
    destroyed -- re-capturing does not accumulate buffers."""
    import ctypes as C
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
    tg = torch.tensor(uniform_targets(512, seed=9), dtype=torch.float64, device=dev)
    q0 = torch.zeros(15, dtype=torch.float64, device=dev)
    out = _bufs(torch, 512, torch.float64, dev)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        s.solve_into(tg, q0, *out, _lib.IKG_F64, side.cuda_stream, check_collision=True)
    torch.cuda.synchronize()
    assert counts(s) == (0, 0)
    held = []
    for k in range(3):  # re-capture three times
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            s.solve_into(tg, q0, *out, _lib.IKG_F64, torch.cuda.current_stream().cuda_stream, check_collision=True)
        g.replay()
        torch.cuda.synchronize()
        live, pend = counts(s)
        assert live >= 1
        held.append(live)
        g.reset()  # destroys the graph and its executable
        import time
        for _ in range(100):  # the user object's destructor may run after the destroy returns
            torch.cuda.synchronize()
            s.solve_into(tg, q0, *out, _lib.IKG_F64, torch.cuda.current_stream().cuda_stream, check_collision=True)
            torch.cuda.synchronize()
            if counts(s) == (0, 0):
                break
            time.sleep(0.02)
        assert counts(s) == (0, 0), (k, counts(s))  # the destroyed graph's scratch was freed
    assert held[0] == held[1] == held[2]
    s.close()
