"""The multi-rank path with the real solver (BASELINE configs[3]):
two ranks share the one GPU of the test box, each solves its contiguous shard
through ikgrasp.parallel.solve_sharded, and the gather to rank 0 equals a
single-rank solve of the whole batch bit for bit.  gloo carries the gather
(host copies) -- the same code runs over RCCL with one rank per GPU."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, dtype, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from ikgrasp.parallel import solve_sharded
    from ikgrasp.solver import IKSolver
    from ikgrasp.workload import uniform_targets
    dist.init_process_group("gloo", rank=rank, world_size=world)
    solver = IKSolver(device=0)
    try:
        tg = uniform_targets(n, seed=77)
        out = solve_sharded(solver, tg, np.zeros(15), dtype=dtype)
        if rank == 0:
            ref = solver.solve(tg, np.zeros(15), dtype=dtype)
            got = {k: v.numpy() for k, v in out.items()}
            q.put(dict(rank=0, world=dist.get_world_size(),
                       q=bool(np.array_equal(got["q"], ref.q)),
                       converged=bool(np.array_equal(got["converged"].astype(bool), ref.converged)),
                       iters=bool(np.array_equal(got["iters"], ref.iters)),
                       err=bool(np.array_equal(got["err"], ref.err)), n=int(got["q"].shape[0])))
        else:
            q.put(dict(rank=rank, none=out is None))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(dict(rank=rank, error=repr(e)))
    finally:
        solver.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("n,dtype", [(4097, "f64"), (2051, "f32")])
def test_two_ranks_on_one_gpu_match_single_rank(n, dtype):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, dtype, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r = q.get(timeout=240)
        res[r["rank"]] = r
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert "error" not in res[0] and "error" not in res[1], res
    assert res[1]["none"]
    r0 = res[0]
    assert r0["world"] == 2 and r0["n"] == n
    assert r0["q"] and r0["converged"] and r0["iters"] and r0["err"], r0
