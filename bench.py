"""Benchmark: grasp-pose IK solves/sec (Nextage dual-arm) on 1..8 MI355X.

    python bench.py [--gpus N --steps K --warmup W --batch B --dtype f64|f32]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step = one launch of the batched IK kernel over this rank's batch of
synthetic grasp targets (already resident in HBM) plus, for N > 1, the RCCL
gather of the final q to rank 0 (north star: "at most an RCCL gather of the
final q over xGMI").  Weak scaling: every rank solves `--batch` targets.
Default workload = BASELINE.json configs[1]: 4,096 targets, fp64, 1 GPU.

`value` counts CONVERGED solves per second over all ranks (the metric's
unit); all problems/s is reported beside it.  The dominant kernel's roofline
is VALU (fp64/fp32 vector ALU, no MFMA, negligible HBM traffic) — see
DESIGN.md §5; the HBM figure the north star asks for is reported as
`roofline_hbm`.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "motion-planning-and-control-for-dual-manipulator-robot_amd"))

METRIC = "grasp-pose IK solves/sec (Nextage dual-arm) at 1/2/4/8 MI355X"
F_ITER = 3144  # FP ops per IK iteration
PEAK_VALU = {"f64": 78.6, "f32": 157.3}  # TFLOP/s vector peaks (MI355X spec)
PEAK_HBM = 8000.0  # GB/s (MI355X_MICROARCH.md)


def algorithmic_bytes(dtype, B, nq=15, broadcast_q0=True):
    """HBM bytes one launch must move: targets + q0 + q + iters + flag + err."""
    s = 8 if dtype == "f64" else 4
    q0 = nq * s if broadcast_q0 else nq * s * B
    return B * (12 * s + nq * s + 4 + 1 + 2 * s) + q0


def multistart_bytes(dtype, T, S, nq=15):
    """Multi-start launch: targets + seeds once, every (target, seed) result
    written to the workspace and its error/flag read back by the best-seed
    reduction, the winner's q read, and the per-target outputs written."""
    s = 8 if dtype == "f64" else 4
    per_problem = (nq * s + 2 * s + 4 + 1) + (2 * s + 1)
    per_target = 12 * s + nq * s + (nq * s + 4 + 1 + 2 * s + 4)
    return T * per_target + S * nq * s + T * S * per_problem


def cpu_baseline(targets, budget_s=10.0):
    """Time the C restatement (oracle/ikg_oracle.c) on host cores over a
    bounded prefix of the same workload."""
    sys.path.insert(0, ROOT)
    from oracle import c_oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    threads = min(threads, 16)
    n_cal = min(len(targets), 8 * threads)
    t0 = time.perf_counter()
    c_oracle.solve(targets[:n_cal], np.zeros(15), threads=threads)
    per = (time.perf_counter() - t0) / n_cal
    # ~budget_s of CPU work: the benchmark targets, repeated as often as needed
    n = int(max(n_cal, budget_s / max(per, 1e-9)))
    reps = -(-n // len(targets))
    sample = np.concatenate([targets] * reps)[:n] if reps > 1 else targets[:n]
    t0 = time.perf_counter()
    _, conv, iters, _ = c_oracle.solve(sample, np.zeros(15), threads=threads)
    dt = time.perf_counter() - t0
    cpu_model = None
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        pass
    return {
        "value": float(conv.sum() / dt), "unit": "converged solves/s", "cores": threads, "kind": "port",
        "cpu_model": cpu_model, "host_cpus": os.cpu_count(),
        "sample": f"{n} solves = the {len(targets)} benchmark targets x {n / len(targets):.2f}, q0=0, fp64 C "
                  f"restatement (oracle/ikg_oracle.c, OpenMP), {dt:.1f} s; all-problem rate {n / dt:.1f}/s",
    }


class QGather:
    """The per-step gather of the final q to rank 0 (north star: "at most an
    RCCL gather of the final q over xGMI").  Device collectives (RCCL): step
    k's gather runs asynchronously on the communicator's stream while step k+1
    solves into the other q buffer; a buffer is handed out again only after
    its gather has been waited on (for RCCL a stream wait, not a host block).
    Host collectives (the gloo rehearsal): synchronous gathers of host copies."""

    def __init__(self, dist, q_out, gathered, world, enabled=True, host=False):
        self.dist, self.gathered, self.host = dist, gathered, host
        self.on = world > 1 and enabled
        self.overlap = self.on and not host
        self.bufs = [q_out, q_out.new_empty(q_out.shape)] if self.overlap else [q_out]
        self.pending = [None] * len(self.bufs)
        self.k = 0

    def buffer(self):
        i = self.k % len(self.bufs)
        if self.pending[i] is not None:
            self.pending[i].wait()
            self.pending[i] = None
        return self.bufs[i]

    def submit(self, qb):
        i = self.k % len(self.bufs)
        assert qb is self.bufs[i]
        self.k += 1
        if not self.on:
            return
        if self.overlap:
            self.pending[i] = self.dist.gather(qb, self.gathered, dst=0, async_op=True)
        else:
            self.dist.gather(qb.cpu() if qb.device.type != "cpu" else qb, self.gathered, dst=0)

    def drain(self):
        for i, w in enumerate(self.pending):
            if w is not None:
                w.wait()
                self.pending[i] = None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="targets per GPU (weak scaling)")
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--yaw", type=float, default=0.0, help="random yaw range (rad) of the cube targets")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--multistart", type=int, default=0,
                    help="seeds per target (BASELINE configs[4]): every target solved from S random seeds, "
                         "best seed kept; value counts converged targets/s")
    ap.add_argument("--collision", action="store_true",
                    help="reference `success` with the collision term (inverse_geometry.py:70, :97-98): "
                         "converged-but-colliding problems iterate on in the continuation kernel; "
                         "value counts collision-free converged solves/s")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # IKG_BENCH_BACKEND=gloo: rehearsal of the multi-rank path on a box with
    # fewer GPUs than ranks (ranks share devices, collectives on host copies);
    # the measured configuration is RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("IKG_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    host = backend != "nccl"  # collectives on host copies

    from ikgrasp import _lib
    from ikgrasp.solver import IKSolver
    from ikgrasp.workload import random_seeds, uniform_targets

    scene = None
    if args.collision:
        from ikgrasp.collision import load_nextage_scene
        scene = load_nextage_scene()
    solver = IKSolver(device=local, scene=scene)
    B = args.batch
    tg_np = uniform_targets(B, seed=rank, yaw=args.yaw)
    tdt = torch.float64 if args.dtype == "f64" else torch.float32
    code = _lib.IKG_F64 if args.dtype == "f64" else _lib.IKG_F32
    targets = torch.tensor(tg_np, dtype=tdt, device=dev)
    q0 = torch.zeros(15, dtype=tdt, device=dev)
    q_out = torch.empty((B, 15), dtype=tdt, device=dev)
    conv = torch.empty(B, dtype=torch.uint8, device=dev)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    err = torch.empty((B, 2), dtype=tdt, device=dev)
    gathered = ([torch.empty_like(q_out, device="cpu" if host else dev) for _ in range(world)]
                if (world > 1 and rank == 0) else None)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    S = args.multistart
    if S:
        seeds_np = random_seeds(solver.model, S, seed=1000 + rank)
        seeds_np[0] = 0.0  # robot.q0 is always one of the seeds
        seeds = torch.tensor(seeds_np, dtype=tdt, device=dev)
        best = torch.empty(B, dtype=torch.int32, device=dev)

    gather = QGather(dist, q_out, gathered, world, enabled=not args.no_gather, host=host)

    def step(ev=None):
        qb = gather.buffer()
        if ev is not None:
            ev[0].record(stream)
        if S:
            solver.solve_multistart_into(targets, seeds, qb, conv, iters, err, best, code, sh,
                                         variant=args.variant, check_collision=args.collision)
        else:
            solver.solve_into(targets, q0, qb, conv, iters, err, code, sh, variant=args.variant,
                              check_collision=args.collision)
        if ev is not None:
            ev[1].record(stream)
        gather.submit(qb)

    for _ in range(args.warmup):
        step()
    gather.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    gather.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))

    n_conv = int(conv.sum().item())
    sum_iters = int(iters.to(torch.int64).sum().item())
    if S:
        # the multi-start launch returns the winner's update count only; its per-seed solves are
        # exactly ikg_solve_batch over the expanded (target, seed) problems (same kernel, same
        # inputs), so one untimed expanded solve gives the updates the timed kernel ran
        n_pr = B * S
        tg_x = targets.repeat_interleave(S, dim=0)
        q0_x = seeds.repeat(B, 1).contiguous()
        q_x = torch.empty((n_pr, 15), dtype=tdt, device=dev)
        c_x = torch.empty(n_pr, dtype=torch.uint8, device=dev)
        i_x = torch.empty(n_pr, dtype=torch.int32, device=dev)
        e_x = torch.empty((n_pr, 2), dtype=tdt, device=dev)
        solver.solve_into(tg_x, q0_x, q_x, c_x, i_x, e_x, code, sh, variant=args.variant,
                          check_collision=args.collision)
        torch.cuda.synchronize()
        sum_iters = int(i_x.to(torch.int64).sum().item())
        del tg_x, q0_x, q_x, c_x, i_x, e_x
    stats = torch.tensor([elapsed, kern_ms, n_conv, B, sum_iters], dtype=torch.float64,
                         device="cpu" if host else dev)
    if world > 1:
        t_max = stats[:2].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        counts = stats[2:].clone()
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
        stats = torch.cat([t_max, counts])
    elapsed, kern_ms, tot_conv, tot_B, tot_iters = stats.tolist()

    # the batch kernel the C-ABI dispatches (ikg_kernels.hip launch_pair_batch): the packed fp32
    # layout from B >= 65,536 on 256 CUs (2 pair waves per SIMD), else the pair layout
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    # (multi-start: AUTO keeps the pair layout)
    packed = args.dtype == "f32" and (args.variant == _lib.IKG_VARIANT_PACKED or
                                      (args.variant == _lib.IKG_VARIANT_AUTO and not S and B > cus * 4 * 32))
    kname = "ikg_packed_batch_kernel" if packed else "ikg_pair_batch_kernel"
    layout = "packed layout (both arms per lane, 64 problems/wave)" if packed else "pair layout (2 lanes/problem)"
    if rank == 0:
        per_step = elapsed / args.steps
        value = tot_conv / per_step
        flops = (sum_iters * F_ITER) / (kern_ms * 1e-3) / 1e12 if sum_iters else None  # rank-0 kernel, TFLOP/s
        abytes = algorithmic_bytes(args.dtype, B) if not S else multistart_bytes(args.dtype, B, S)
        traffic = None
        pmc = os.path.join(ROOT, "profiles", f"pmc_{args.dtype}_b{B}.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        # executed FP ops per problem-iteration of this kernel (rocprofv3 FMA/MUL/ADD/TRANS counters,
        # tools/pmc_flops.py): the frame-1 loop does ~1/3 of the reference formulation's 3,144, so the
        # SURVEY-count frac above overstates hardware use; executed_frac is the hardware VALU fraction
        executed = None
        fl = os.path.join(ROOT, "profiles", f"flops_{args.dtype}_b{B}.json")
        if os.path.exists(fl) and kname == "ikg_pair_batch_kernel" and sum_iters:
            with open(fl) as f:
                per_it = json.load(f)["fp_ops_per_problem_iter"]
            ex = sum_iters * per_it / (kern_ms * 1e-3) / 1e12
            waves = -(-B // 32)
            executed = {"fp_ops_per_problem_iter": per_it, "achieved": ex, "frac": ex / PEAK_VALU[args.dtype],
                        "unit": "TFLOP/s", "waves": waves, "simds": cus * 4,
                        "source": os.path.relpath(fl, ROOT)}
        out = {
            "metric": METRIC, "value": value, "unit": "converged solves/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": per_step * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (cube targets ~ path.py:35-47 sampler, seed = rank; q0 = robot.q0 = 0)",
            "config": {
                "workload": (f"BASELINE configs[4]: multi-start {S} seeds x {B} targets per GPU, {args.dtype}"
                             if S else
                             f"BASELINE configs[1]: batch {B} grasp targets per GPU, {args.dtype}, "
                             f"{layout}") +
                            (" + collision term (continuation kernel)" if args.collision else ""),
                "collision_term": bool(args.collision),
                "seeds_per_target": S or 1,
                "batch_per_gpu": B, "global_batch": B * world, "yaw_range": args.yaw,
                "parallelism": f"shard{world}" + ("" if world == 1 or args.no_gather else
                                                  ("+rccl_gather_q" if not host else "+gloo_gather_q")),
            },
            "problems_per_s": tot_B / per_step,
            "converged_fraction": tot_conv / tot_B,
            "mean_iters": (tot_iters / tot_B) if not S else None,
            "mean_iters_all_problems": (tot_iters / (tot_B * S)) if S else None,
            "roofline": {
                "bound": "valu", "achieved": flops, "peak": PEAK_VALU[args.dtype], "unit": "TFLOP/s",
                "frac": flops / PEAK_VALU[args.dtype] if flops else None, "traffic": traffic,
                "kernel": kname + (" + ikg_collide_continue_kernel" if args.collision else ""),
                "kernel_ms": kern_ms,
                "work": f"sum(iters)={sum_iters} x {F_ITER} FP ops (SURVEY §8a)",
                "executed": executed,
            },
            "roofline_hbm": {
                "bound": "hbm", "achieved": abytes / (kern_ms * 1e-3) / 1e9, "peak": PEAK_HBM, "unit": "GB/s",
                "frac": abytes / (kern_ms * 1e-3) / 1e9 / PEAK_HBM, "traffic": traffic,
                "algorithmic_bytes": abytes,
            },
        }
        if world == 1 and not args.no_cpu_baseline and not S and not args.collision:
            out["cpu_baseline"] = cpu_baseline(tg_np)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    solver.close()


if __name__ == "__main__":
    main()
