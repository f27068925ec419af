"""Multi-GPU sharding of a grasp-target batch.

Problems are independent, so a batch is split into contiguous per-rank
slices, each rank solves its slice on its own GPU, and (optionally) the final
q / flags are gathered to the root over RCCL.  Multi-start shards targets,
never seeds, so the best-seed reduction stays on one GPU.  No other
collective exists on this path.
"""
from __future__ import annotations


def shard_range(n: int, rank: int, world: int):
    """Contiguous balanced slice [lo, hi) of n items for `rank` of `world`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_sizes(n: int, world: int):
    return [shard_range(n, r, world)[1] - shard_range(n, r, world)[0] for r in range(world)]


def gather_rows(local, n_total: int, dst: int = 0, group=None):
    """Gather per-rank row blocks (equal or ±1 rows) to `dst`; returns the
    concatenated [n_total, ...] tensor on dst and None elsewhere.

    Uneven shards are padded to the largest shard so a single collective
    (`torch.distributed.gather`; RCCL on ROCm devices, gloo on CPU) moves
    everything.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = shard_sizes(n_total, world)
    cap = max(sizes)
    if local.shape[0] != sizes[rank]:
        raise ValueError(f"rank {rank}: local rows {local.shape[0]} != shard size {sizes[rank]}")
    if local.shape[0] < cap:
        pad = torch.zeros((cap - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        send = torch.cat([local, pad])
    else:
        send = local.contiguous()
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)])


def solve_sharded(solver, targets, q0, dtype="f64", dst=0, **kw):
    """Solve a global batch across all ranks (config C4): rank r solves its
    slice of `targets` (a host array, identical on every rank) on its device
    and q / converged / iters / err are gathered to `dst`."""
    import numpy as np
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    lo, hi = shard_range(len(targets), rank, world)
    dev = torch.device("cuda", solver.device)
    tdt = torch.float64 if dtype == "f64" else torch.float32
    tg = torch.tensor(np.asarray(targets[lo:hi]), dtype=tdt, device=dev)
    q = torch.as_tensor(np.asarray(q0), dtype=tdt, device=dev)
    if q.dim() == 2:
        q = q[lo:hi]
    sol = solver.solve(tg, q, **kw)
    host = dist.get_backend() == "gloo"  # gloo gathers host tensors (the rehearsal of RCCL's device gather)
    out = {}
    for name, t in (("q", sol.q), ("converged", sol.converged.to(torch.uint8)), ("iters", sol.iters),
                    ("err", sol.err)):
        out[name] = gather_rows(t.cpu() if host else t, len(targets), dst=dst)
    return out if rank == dst else None
