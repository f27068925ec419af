"""Multi-rank path on CPU: shard arithmetic and the root gather over gloo at
world size 2 (the GPU path uses the same code over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ikgrasp.parallel import gather_rows, shard_range, shard_sizes


@pytest.mark.parametrize("n,world", [(10, 2), (11, 2), (4096, 8), (1, 2), (0, 2), (1048576, 8)])
def test_shards_cover_exactly(n, world):
    covered = []
    for r in range(world):
        lo, hi = shard_range(n, r, world)
        covered.extend(range(lo, hi))
    assert covered == list(range(n))
    assert max(shard_sizes(n, world)) - min(shard_sizes(n, world)) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.arange(n * 15, dtype=torch.float64).reshape(n, 15)
        lo, hi = shard_range(n, rank, world)
        local = full[lo:hi] * 2.0  # stand-in for the per-rank solve
        flags = (torch.arange(lo, hi) % 3 == 0).to(torch.uint8)
        g = gather_rows(local, n)
        gf = gather_rows(flags, n)
        if rank == 0:
            q.put((torch.equal(g, full * 2.0), torch.equal(gf, (torch.arange(n) % 3 == 0).to(torch.uint8))))
        else:
            q.put((g is None, gf is None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [10, 7])
def test_gather_rows_world2_gloo(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(a and b for a, b in res)


def _qgather_worker(rank, world, port, host, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import QGather

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q_out = torch.zeros(6, 15, dtype=torch.float64)
        gathered = [torch.empty_like(q_out) for _ in range(world)] if rank == 0 else None
        g = QGather(dist, q_out, gathered, world, enabled=True, host=host)
        ids, ok = [], True
        for k in range(5):  # bench.py's step(): buffer -> solve into it -> submit
            qb = g.buffer()
            ok &= all(w is None for i, w in enumerate(g.pending) if g.bufs[i] is qb)
            ids.append(id(qb))
            qb.fill_(10.0 * k + rank)
            g.submit(qb)
        g.drain()
        ok &= all(w is None for w in g.pending)
        alternates = len(set(ids)) == (1 if host else 2) and all(ids[i] == ids[i % len(g.bufs)] for i in range(5))
        if rank == 0:
            out = g.result()
            ok &= all(torch.all(out[r] == 40.0 + r).item() for r in range(world))
        q.put((rank, ok and alternates))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("host", [False, True])
def test_bench_gather_pipeline_world2_gloo(host):
    """bench.py's per-step q gather: the overlapped double-buffered form (the
    RCCL path; async gathers) and the synchronous host-copy form deliver the
    last step's q of every rank to rank 0, and a buffer is never handed out
    while its gather is in flight."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_qgather_worker, args=(r, 2, port, host, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res), res
