"""Benchmark: grasp-pose IK solves/sec (Nextage dual-arm) on 1..8 MI355X.

    python bench.py [--gpus N --steps K --warmup W --batch B --dtype f64|f32]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`--gpus N > 1` without a launcher (WORLD_SIZE unset) starts the N rank
processes itself (a child `torch.distributed.run`, one rank per GPU); with
fewer GPUs than ranks it rehearses over gloo (ranks share the devices,
collectives on host copies) and says so in `config.parallelism`.

A step = one launch of the batched IK kernel over this rank's batch of
synthetic grasp targets (already resident in HBM) plus, for N > 1, the RCCL
gather of the final q to rank 0 (north star: "at most an RCCL gather of the
final q over xGMI").  Weak scaling: every rank solves `--batch` targets.
Default workload = BASELINE.json configs[1]: 4,096 targets, fp64.

`value` counts CONVERGED solves per second over all ranks (the metric's
unit); all problems/s is reported beside it.  The dominant kernel's roofline
is VALU (fp64/fp32 vector ALU, no MFMA, negligible HBM traffic) — see
DESIGN.md §5; the HBM figure the north star asks for is `roofline_hbm`.

The same JSON line carries, under `extra` (timed after the headline):
  * `c4_strong`: BASELINE configs[3], 1,048,576 targets split over the ranks
    (strong scaling), each step the shard solves plus the RCCL gather of q,
    flags and update counts to rank 0 (ikgrasp.parallel);
  * `c2_collision`: configs[1] with the reference's `success` (the collision
    term of inverse_geometry.py:70, :97-98), with its own roofline and CPU leg;
  * `c2_yaw`: configs[1] with random cube yaw in [-pi/4, pi/4] (the "random
    SE(3)" reading), with its own roofline and CPU leg.
Every roofline block carries the executed-FP-ops fraction beside the
SURVEY-count one, and a note wherever the SURVEY-count fraction exceeds 1.
Multi-rank lines carry `ranks`: per-rank kernel ms and the gather's own ms.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "motion-planning-and-control-for-dual-manipulator-robot_amd"))

METRIC = "grasp-pose IK solves/sec (Nextage dual-arm) at 1/2/4/8 MI355X"
F_ITER = 3144  # FP ops per IK iteration of the reference formulation
# Vector (VALU) peaks, TFLOP/s: fp32 from MI355X_MICROARCH.md (157.3); fp64 is
# AMD's MI355X spec-sheet figure (78.6), not listed in the guide
PEAK_VALU = {"f64": 78.6, "f32": 157.3}
PEAK_HBM = 8000.0  # GB/s (MI355X_MICROARCH.md)
C4_TOTAL = 1 << 20  # BASELINE configs[3]


# ---------------------------------------------------------------- host / CPU
def cpu_share():
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU
    quota (the GPU box gives a job a share of a large host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(p)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                p = int(f.read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    return max(1, min(n, int(quota)) if quota else n), quota


def host_cpus():
    """(model name, logical CPUs, physical cores) of the host."""
    model, cores = None, set()
    phys = core = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                k, _, v = ln.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and model is None:
                    model = v
                elif k == "physical id":
                    phys = v
                elif k == "core id":
                    core = v
                elif not k and phys is not None and core is not None:
                    cores.add((phys, core))
                    phys = core = None
    except OSError:
        pass
    if phys is not None and core is not None:
        cores.add((phys, core))
    return model, os.cpu_count(), len(cores) or None


def cpu_baseline(targets, budget_s=10.0, numpy_budget_s=8.0):
    """The reference-semantics CPU loop on this host, beside the GPU run:
    (1) the C restatement (oracle/ikg_oracle.c, OpenMP, one problem per
    thread) on every CPU this job may use, ~budget_s of work over the
    benchmark's own targets (repeated); (2) the numpy oracle
    (oracle/ik_oracle.py: the reference-shaped loop, np.linalg.pinv) on one
    core over a prefix of the targets.  The host's full core count is stated
    with a per-core extrapolation; the measured value is what ran."""
    sys.path.insert(0, ROOT)
    from oracle import c_oracle, ik_oracle
    threads, quota = cpu_share()
    if os.environ.get("IKG_CPU_THREADS"):
        threads = int(os.environ["IKG_CPU_THREADS"])
    n_cal = min(len(targets), 8 * threads)
    t0 = time.perf_counter()
    c_oracle.solve(targets[:n_cal], np.zeros(15), threads=threads)
    per = (time.perf_counter() - t0) / n_cal
    n = int(max(n_cal, budget_s / max(per, 1e-9)))
    reps = -(-n // len(targets))
    sample = np.concatenate([targets] * reps)[:n] if reps > 1 else targets[:n]
    t0 = time.perf_counter()
    _, conv, iters, _ = c_oracle.solve(sample, np.zeros(15), threads=threads)
    dt = time.perf_counter() - t0
    model, logical, physical = host_cpus()
    value = float(conv.sum() / dt)
    # numpy single core: whole solves until the budget is spent
    t0, k, nconv = time.perf_counter(), 0, 0
    while time.perf_counter() - t0 < numpy_budget_s and k < len(targets):
        t = targets[k]
        _, ok, _, _ = ik_oracle.computeqgrasppose(np.zeros(15), t[:9].reshape(3, 3), t[9:])
        nconv += bool(ok)
        k += 1
    dn = max(time.perf_counter() - t0, 1e-9)
    return {
        "value": value, "unit": "converged solves/s", "cores": threads, "kind": "port",
        "sample": f"{n} solves = the {len(targets)} benchmark targets x {n / len(targets):.2f}, q0=0, fp64 C "
                  f"restatement (oracle/ikg_oracle.c, OpenMP, {threads} threads), {dt:.1f} s; "
                  f"all-problem rate {n / dt:.1f}/s",
        "cpu_model": model, "host_logical_cpus": logical, "host_physical_cores": physical,
        "job_cpu_share": quota, "threads_used": threads,
        "per_thread_converged_per_s": value / threads,
        "all_physical_cores_extrapolated": (value / threads * physical) if physical else None,
        "numpy_single_core": None if k == 0 else {
            "value": nconv / dn, "unit": "converged solves/s", "cores": 1, "kind": "port",
            "sample": f"first {k} benchmark targets, oracle/ik_oracle.py (np.linalg.pinv per update), {dn:.1f} s, "
                      f"{nconv} converged; {k / dn:.2f} problems/s"},
    }


def cpu_baseline_collision(targets, scene_json, budget_s=8.0):
    """The reference-semantics loop WITH the collision term (the C collision
    restatement in oracle/ikg_oracle.c, checked against
    tests/golden/collision_cases.npz), on every CPU this job may use, over
    the same scene the GPU run uses."""
    sys.path.insert(0, ROOT)
    from oracle import c_oracle, collision_oracle
    if not c_oracle.has_collision():
        return None
    sc = collision_oracle.prepare(json.loads(scene_json))
    threads, _ = cpu_share()
    if os.environ.get("IKG_CPU_THREADS"):
        threads = int(os.environ["IKG_CPU_THREADS"])
    n_cal = min(len(targets), 4 * threads)
    t0 = time.perf_counter()
    c_oracle.solve_collision(sc, targets[:n_cal], np.zeros(15), threads=threads)
    per = (time.perf_counter() - t0) / n_cal
    n = int(max(n_cal, budget_s / max(per, 1e-9)))
    reps = -(-n // len(targets))
    sample = np.concatenate([targets] * reps)[:n] if reps > 1 else targets[:n]
    t0 = time.perf_counter()
    _, ok, _, _ = c_oracle.solve_collision(sc, sample, np.zeros(15), threads=threads)
    dt = time.perf_counter() - t0
    return {"value": float(ok.sum() / dt), "unit": "collision-free converged solves/s", "cores": threads,
            "kind": "port",
            "sample": f"{n} solves of the benchmark targets, q0=0, fp64 C restatement with the collision term "
                      f"(oracle/ikg_oracle.c), {dt:.1f} s"}


# ---------------------------------------------------------------- roofline inputs
def flops_profile(kernel, dtype, med):
    """Executed FP operations per problem-update of a kernel (rocprofv3 VALU
    instruction counters, tools/pmc_flops.py) -> (ops, source) or None."""
    names = [f"flops_{kernel}_{dtype}{'_med' if med else ''}.json"]
    if kernel == "pair" and not med:
        names.append(f"flops_{dtype}_b4096.json")  # round-2 name
    for n in names:
        p = os.path.join(ROOT, "profiles", n)
        if os.path.exists(p):
            with open(p) as f:
                return json.load(f)["fp_ops_per_problem_iter"], os.path.relpath(p, ROOT)
    return None


def hbm_profile(dtype, B, S=0, collision=False, variant=""):
    """Counter HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE) for this
    configuration, from profiles/pmc_*.json, or None."""
    tag = (f"pmc_{dtype}_b{B}" + (f"_s{S}" if S else "") + ("_col" if collision else "") +
           (f"_{variant}" if variant else "") + ".json")
    p = os.path.join(ROOT, "profiles", tag)
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f).get("hbm_bytes_per_launch"), os.path.relpath(p, ROOT)
    return None, None


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


SHADER_GHZ = 2.4  # MI355X peak engine clock (MI355X_MICROARCH.md): used only without a measured clock


def measured_clock(kernel, dtype):
    """The in-kernel shader clock the stage-stamp build measured on this
    kernel (tools/stage_clock.py: Δs_memtime / Δs_memrealtime x 100 MHz over
    every wave's loop, after >= 2 s of back-to-back launches) -> (GHz, source)."""
    p = os.path.join(ROOT, "profiles", f"stage_{kernel}_{dtype}.json")
    if os.path.exists(p):
        with open(p) as f:
            d = json.load(f)
        ghz = (d.get("c2") or d.get("forced") or {}).get("clock_GHz")
        if ghz:
            return ghz, os.path.relpath(p, ROOT), d
    return SHADER_GHZ, "assumed peak engine clock (MI355X_MICROARCH.md)", None


def latency_block(kernel, dtype, med, kern_ms, max_iters, waves, simds):
    """The bound that actually binds a launch with at most one wave per SIMD:
    one wave's in-order issue of an update's instruction stream, times the
    updates of the longest-running wave.  Per-update cycles come from the
    committed ISA model (tools/isa_critpath.py: the hot loop's instructions
    issued in order, a VALU op at most every 4 cycles, each waiting for its
    operands at the measured gfx950 latencies), the updates and the kernel
    time from this run."""
    p = os.path.join(ROOT, "profiles", f"latency_{kernel}_{dtype}{'_med' if med else ''}.json")
    if not os.path.exists(p) or not max_iters or waves > simds:
        return None
    with open(p) as f:
        m = json.load(f)
    ghz, clk_src, stage = measured_clock(kernel, dtype)
    pred = max_iters * m["in_order_cycles"] / (ghz * 1e6)
    out = {
        "bound": "per-wave in-order issue of one update's dependent instruction stream (waves <= SIMDs)",
        "updates_longest_wave": max_iters,
        "instructions_per_update": m["instructions_per_update"], "valu_per_update": m["valu_per_update"],
        "issue_bound_cycles_per_update": m["issue_bound_cycles"],
        "critical_path_cycles_per_update": m["critical_path_cycles"],
        "model_cycles_per_update": m["in_order_cycles"], "stall_cycles_per_update": m["stall_cycles"],
        "register_copies_per_update": m.get("register_copies_per_update"),
        "clock_GHz": ghz, "clock_source": clk_src, "predicted_ms": pred, "measured_ms": kern_ms,
        "measured_cycles_per_update": kern_ms * ghz * 1e6 / max_iters,
        "frac": pred / kern_ms, "source": os.path.relpath(p, ROOT),
    }
    if stage and stage.get("forced"):
        f = stage["forced"]
        out["stages_measured"] = {
            "cycles_per_update_each_stage_alone": f["diag_stage_cycles_per_update"],
            "stamped_loop_cycles_per_update": f["diag_loop_cycles_per_update"],
            "is": "s_memtime stamps between the stages (diagnostic build, every lane runs 1,000 updates); "
                  "fenced stages cannot overlap, so they sum above the product loop's cycles"}
    return out


def roofline(dtype, kernel, med, kern_ms, sum_iters, waves, simds, abytes, traffic, traffic_src, max_iters=None):
    """The dominant kernel's VALU roofline (SURVEY count and executed count)
    and its HBM figures (algorithmic bytes and counter bytes), for ONE GPU:
    `sum_iters`, `waves`, `abytes` and `traffic` are that GPU's, `kern_ms` its
    kernel time."""
    survey = (sum_iters * F_ITER) / (kern_ms * 1e-3) / 1e12 if sum_iters else None
    ex = flops_profile(kernel, dtype, med)
    executed = None
    if ex and sum_iters:
        a = sum_iters * ex[0] / (kern_ms * 1e-3) / 1e12
        executed = {"fp_ops_per_problem_iter": ex[0], "achieved": a, "frac": a / PEAK_VALU[dtype],
                    "unit": "TFLOP/s", "waves": waves, "simds": simds, "source": ex[1]}
    frac = survey / PEAK_VALU[dtype] if survey else None
    out = {
        "bound": "valu", "achieved": survey, "peak": PEAK_VALU[dtype], "unit": "TFLOP/s", "frac": frac,
        "traffic": traffic, "kernel_ms": kern_ms,
        "work": f"sum(updates)={sum_iters} x {F_ITER} FP ops (SURVEY §8a reference formulation)",
        "executed": executed,
    }
    if frac and frac > 1:
        out["note"] = ("frac > 1: the kernel's closed-form frame-1 loop executes fewer FP ops than the "
                       "reference formulation it is priced at (see executed)")
    lat = latency_block(kernel, dtype, med, kern_ms, max_iters, waves, simds)
    if lat:
        out["latency"] = lat
    hbm = {"bound": "hbm", "algorithmic_bytes": abytes,
           "algorithmic_GBps": abytes / (kern_ms * 1e-3) / 1e9, "peak": PEAK_HBM, "unit": "GB/s",
           "traffic": traffic, "traffic_source": traffic_src}
    if traffic:
        hbm["achieved"] = traffic / (kern_ms * 1e-3) / 1e9
        hbm["frac"] = hbm["achieved"] / PEAK_HBM
    else:
        hbm["achieved"] = hbm["algorithmic_GBps"]
        hbm["frac"] = hbm["achieved"] / PEAK_HBM
        hbm["achieved_is"] = "algorithmic bytes (no counter profile for this configuration)"
    return out, hbm


def iters_hist(iters, max_iters=1000, width=50):
    """Update-count histogram (SURVEY §5 "Metrics"; the reference's own
    convergence evidence is per-iteration charts, inverse_geometry_TESTS.py:403-450):
    50-update bins [lo, lo + 49] below max_iters, and the max_iters bucket (the
    loop exhausted: not converged, or converged-but-colliding that ran on)."""
    it = np.asarray(iters).astype(np.int64).ravel()
    h = {}
    for lo in range(0, max_iters, width):
        h[f"{lo}-{min(lo + width, max_iters) - 1}"] = int(((it >= lo) & (it < lo + width) & (it < max_iters)).sum())
    h[str(max_iters)] = int((it >= max_iters).sum())
    return h


REC_BUDGET_MB, CK_BUDGET_MB = 1024, 16384  # ikg_capi.hip kRecBudgetMB / kCkBudgetMB (IKG_REC_BUDGET_MB / IKG_CK_BUDGET_MB)


def collision_kernels(kname, dtype, B, S=0):
    """The kernels a collision solve runs, by the C-ABI's rules
    (ikg_capi.hip rec_chunk / offer_records, ikg_collision.hip
    launch_collide_continue): the batch kernel writing window checkpoints, in
    launches whose checkpoints fit their budget; then per launch the first
    check (the pre-screen, then the window-box tests over its list; fused with
    IKG_PRESCAN=1), and per records round the resume launch of the batch kernel
    (windows left) and the records scan."""
    esz = 8 if dtype == "f64" else 4
    ck = esz * 64 * (1000 // 32 + 3) * max(S, 1)  # one unit's checkpoints (a target's S seeds)
    rec = esz * 20 * 1001  # one listed problem's records
    budget = int(os.environ.get("IKG_CK_BUDGET_MB", str(CK_BUDGET_MB))) << 20
    cap = max(1, budget // ck)
    chunks = 1 if B <= cap else -(-B // cap)
    per = -(-B // chunks) * max(S, 1)  # problems per launch
    slots = max(1, (int(os.environ.get("IKG_REC_BUDGET_MB", str(REC_BUDGET_MB))) << 20) // rec)
    rounds = -(-per // min(per, slots))
    fused = os.environ.get("IKG_PRESCAN", "0") != "0"
    label = (kname + " (window checkpoints past the first passing iterate) + " +
             ("ikg_first_check_kernel (first check and window boxes, one wave per problem)" if fused else
              "ikg_prescreen_kernel (first check, lists the colliding) + ikg_first_check_kernel (window boxes "
              "over its list)") +
             " + " + kname + f" (resume: windows left) + ikg_traj_scan_kernel (records scan, up to 8 waves per "
             f"listed problem), {rounds} records round(s)")
    if chunks > 1:
        label += f"; {chunks} launch sequences of {per} problems (checkpoint budget {budget >> 20} MB)"
    return label, "the whole solve (all its kernels)"


# ---------------------------------------------------------------- launcher
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """--gpus N without a launcher: N rank processes under a child
    torch.distributed.run (not an exec of this process).  Fewer GPUs than
    ranks: a gloo rehearsal (ranks share devices; not a throughput number)."""
    import torch
    env = dict(os.environ)
    ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
    if ndev < n and "IKG_BENCH_BACKEND" not in env:
        env["IKG_BENCH_BACKEND"] = "gloo"
        print(f"[bench] {n} ranks on {ndev} GPU(s): gloo rehearsal", file=sys.stderr)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------- GPU side
class QGather:
    """The per-step gather of the final q to rank 0 (north star: "at most an
    RCCL gather of the final q over xGMI").  Device collectives (RCCL): step
    k's gather runs asynchronously on the communicator's stream while step k+1
    solves into the other q buffer; a buffer is handed out again only after
    its gather has been waited on (for RCCL a stream wait, not a host block).
    Host collectives (the gloo rehearsal): synchronous gathers of host copies."""

    def __init__(self, dist, q_out, gathered, world, enabled=True, host=False):
        self.dist, self.host = dist, host
        self.on = world > 1 and enabled
        self.overlap = self.on and not host
        self.bufs = [q_out, q_out.new_empty(q_out.shape)] if self.overlap else [q_out]
        # rank 0's outputs are double-buffered with the inputs: two gathers in
        # flight never write the same tensors, whatever order the backend
        # completes them in (gloo runs async work on several threads)
        self.outs = [gathered] + ([[t.new_empty(t.shape) for t in gathered]] if self.overlap and gathered else
                                  [gathered] * (len(self.bufs) - 1))
        self.pending = [None] * len(self.bufs)
        self.k = 0

    def result(self):
        """rank 0: the last submitted step's gathered q (after drain())."""
        return self.outs[(self.k - 1) % len(self.bufs)]

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
            self.pending[i] = self.dist.gather(qb, self.outs[i], dst=0, async_op=True)
        else:
            self.dist.gather(qb.cpu() if qb.device.type != "cpu" else qb, self.outs[i], dst=0)

    def drain(self):
        for i, w in enumerate(self.pending):
            if w is not None:
                w.wait()
                self.pending[i] = None


def timed(torch, dist, world, steps, warmup, step, stream, drain=None):
    """warmup untimed steps, then `steps` timed ones bracketed by a barrier
    and synchronize; returns (this rank's wall s, mean kernel ms) where the
    kernel time is HIP events on the launch stream around each solve.
    `drain` completes outstanding collectives inside the timed region."""
    for _ in range(warmup):
        step(None)
    if drain:
        drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for k in range(steps):
        step(events[k])
    if drain:
        drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    return elapsed, float(np.mean([a.elapsed_time(b) for a, b in events]))


def reduce_stats(torch, dist, world, host, dev, vals, n_max):
    """[max over ranks of the first n_max values] + [sum of the rest]."""
    t = torch.tensor(vals, dtype=torch.float64, device="cpu" if host else dev)
    if world > 1:
        mx = t[:n_max].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t[n_max:].clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        t = torch.cat([mx, sm])
    return t.tolist()


def per_rank(torch, dist, world, host, dev, vals):
    """Every rank's `vals` (a few floats) -> [world][len(vals)] on every rank."""
    t = torch.tensor(vals, dtype=torch.float64, device="cpu" if host else dev)
    if world == 1:
        return [t.tolist()]
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def time_collective(torch, dist, world, fn, reps=5):
    """Mean wall ms of one blocking collective step `fn()`, each repetition
    started from a barrier with the device idle and ended by a device
    synchronize (untimed by the step loop: the diagnosable share of a step)."""
    if world == 1:
        return None
    ms = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
    return float(np.mean(ms[1:]))


def rank_block(per, world, backend, gather_ms, what):
    """The per-rank figures of a multi-rank run (first diagnosis of an 8-GPU line)."""
    km = [r[0] for r in per]
    return {"world_size_seen": world, "backend": backend if world > 1 else None,
            "kernel_ms_per_rank": km, "kernel_ms_min": min(km), "kernel_ms_max": max(km),
            "gather_ms": gather_ms, "gather_is": what if world > 1 else "no collective at N=1"}


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
    ap.add_argument("--no-extra", action="store_true", help="skip the c4_strong / c2_collision extras")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--multistart", type=int, default=0,
                    help="seeds per target (BASELINE configs[4]): every target solved from S random seeds, "
                         "best seed kept; value counts converged targets/s")
    ap.add_argument("--collision", action="store_true",
                    help="reference `success` with the collision term (inverse_geometry.py:70, :97-98) as the "
                         "headline; value counts collision-free converged solves/s")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    # stdout carries exactly one line, the JSON result: everything else the
    # libraries print there (gloo's peer-connection notices, RCCL / HIP chatter)
    # is sent to stderr, and the result is written to the saved stdout
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # IKG_BENCH_BACKEND=gloo: rehearsal of the multi-rank path on a box with
    # fewer GPUs than ranks (ranks share devices, collectives on host copies);
    # the measured configuration is RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("IKG_BENCH_BACKEND", "nccl")
    ndev = max(1, torch.cuda.device_count())
    if backend == "gloo":
        local = local % ndev
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()  # what the communicator saw
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    host = backend != "nccl"  # collectives on host copies

    from ikgrasp import _lib
    from ikgrasp.collision import load_nextage_scene
    from ikgrasp.parallel import gather_rows, shard_range
    from ikgrasp.solver import IKSolver
    from ikgrasp.workload import random_seeds, uniform_targets

    solver = IKSolver(device=local, scene=load_nextage_scene())
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

    def step(ev):
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

    elapsed, kern_ms = timed(torch, dist, world, args.steps, args.warmup, step, stream, drain=gather.drain)
    per = per_rank(torch, dist, world, host, dev, [kern_ms])

    def gather_once():
        if host:
            dist.gather(q_out.cpu(), gathered, dst=0)
        else:
            dist.gather(q_out, gathered, dst=0)
    gather_ms = time_collective(torch, dist, world, gather_once) if (world > 1 and not args.no_gather) else None

    n_conv = int(conv.sum().item())
    sum_iters = int(iters.to(torch.int64).sum().item())
    max_iters = int(iters.max().item()) if B else 0
    hist = iters_hist(iters.cpu().numpy())
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
        hist = iters_hist(i_x.cpu().numpy())
        del tg_x, q0_x, q_x, c_x, i_x, e_x
    elapsed, kern_ms, tot_conv, tot_B, tot_iters = reduce_stats(
        torch, dist, world, host, dev, [elapsed, kern_ms, n_conv, B, sum_iters], 2)

    # the batch kernel the C-ABI dispatches (ikg_kernels.hip launch_pair_batch): the packed fp32
    # layout from B >= 65,536 on 256 CUs (2 pair waves per SIMD), else the pair layout
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    packed = args.dtype == "f32" and (args.variant == _lib.IKG_VARIANT_PACKED or
                                      (args.variant == _lib.IKG_VARIANT_AUTO and not S and B > cus * 4 * 32))
    kname = "ikg_packed_batch_kernel" if packed else "ikg_pair_batch_kernel"
    layout = "packed layout (both arms per lane, 64 problems/wave)" if packed else "pair layout (2 lanes/problem)"
    ppw = 64 if packed else 32

    extra = {}
    if not args.no_extra and not S and not args.collision:
        extra = run_extras(torch, dist, world, rank, host, dev, solver, code, tdt, args, stream, sh, gather_rows,
                           shard_range, uniform_targets)

    if rank == 0:
        per_step = elapsed / args.steps
        value = tot_conv / per_step
        abytes = algorithmic_bytes(args.dtype, B) if not S else multistart_bytes(args.dtype, B, S)
        traffic, tsrc = hbm_profile(args.dtype, B, S, args.collision)
        rl, rl_hbm = roofline(args.dtype, "packed" if packed else "pair", bool(S), kern_ms, sum_iters,
                              -(-B * max(S, 1) // ppw), cus * 4, abytes, traffic, tsrc,
                              max_iters=None if (S or args.collision) else max_iters)
        if args.collision:
            rl["kernel"], rl["kernel_ms_covers"] = collision_kernels(kname, args.dtype, B, S)
        else:
            rl["kernel"] = kname
        parallelism = f"shard{world}"
        if world > 1:
            parallelism += "" if args.no_gather else ("+rccl_gather_q" if not host else "+gloo_gather_q")
            if host:
                parallelism += " (gloo rehearsal: ranks share GPUs, not a throughput number)"
        out = {
            "metric": METRIC, "value": value, "unit": "converged solves/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": per_step * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (cube targets ~ path.py:35-47 sampler, seed = rank; q0 = robot.q0 = 0)",
            "config": {
                "workload": (f"BASELINE configs[4]: multi-start {S} seeds x {B} targets per GPU, {args.dtype}"
                             if S else
                             f"BASELINE configs[1]: batch {B} grasp targets per GPU, {args.dtype}, {layout}") +
                            (" + collision term" if args.collision else ""),
                "collision_term": bool(args.collision),
                "seeds_per_target": S or 1,
                "batch_per_gpu": B, "global_batch": B * world, "yaw_range": args.yaw,
                "parallelism": parallelism, "world_size_seen": world, "backend": backend if world > 1 else None,
                "devices_visible": ndev,
            },
            "problems_per_s": tot_B / per_step,
            "converged_fraction": tot_conv / tot_B,
            "mean_iters": (tot_iters / tot_B) if not S else None,
            "mean_iters_all_problems": (tot_iters / (tot_B * S)) if S else None,
            "iters_hist": hist,
            "iters_hist_is": ("update counts of every (target, seed) problem of rank 0's launch" if S else
                              "update counts of rank 0's batch") + " (50-update bins; '1000': the loop exhausted)",
            "roofline": rl,
            "roofline_hbm": rl_hbm,
            "ranks": rank_block(per, world, backend, gather_ms,
                                f"blocking dist.gather of one step's q ({B}x15 {args.dtype}) to rank 0, wall ms"),
        }
        if world == 1 and not args.no_cpu_baseline and not S and not args.collision:
            out["cpu_baseline"] = cpu_baseline(tg_np)
        if "c2_collision" in extra:  # the reference's success (collision term) beside the headline's
            out["value_with_collision"] = extra["c2_collision"]["value"]
            out["value_with_collision_is"] = ("extra.c2_collision: collision-free converged solves/s, the "
                                              "reference's success (inverse_geometry.py:70, :97-98)")
        if extra:
            if world == 1 and not args.no_cpu_baseline and "c2_collision" in extra:
                extra["c2_collision"]["cpu_baseline"] = cpu_baseline_collision(tg_np, solver.scene.to_json())
            out["extra"] = extra
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if world > 1:
        dist.destroy_process_group()
    solver.close()


def run_extras(torch, dist, world, rank, host, dev, solver, code, tdt, args, stream, sh, gather_rows, shard_range,
               uniform_targets):
    """The c4_strong and c2_collision figures (see the module docstring)."""
    from ikgrasp import _lib
    extra = {}
    # ---- C4: 1,048,576 targets split over the ranks, gather of q / flags / iters to rank 0
    tot = C4_TOTAL
    lo, hi = shard_range(tot, rank, world)
    all_t = uniform_targets(tot, seed=7)
    n = hi - lo
    tg4 = torch.tensor(all_t[lo:hi], dtype=torch.float64, device=dev)
    del all_t
    q04 = torch.zeros(15, dtype=torch.float64, device=dev)
    q4 = torch.empty((n, 15), dtype=torch.float64, device=dev)
    c4 = torch.empty(n, dtype=torch.uint8, device=dev)
    i4 = torch.empty(n, dtype=torch.int32, device=dev)
    e4 = torch.empty((n, 2), dtype=torch.float64, device=dev)

    def gather4():
        for t in (q4, c4, i4):
            gather_rows(t.cpu() if host else t, tot, dst=0)

    def step4(ev):
        if ev is not None:
            ev[0].record(stream)
        solver.solve_into(tg4, q04, q4, c4, i4, e4, _lib.IKG_F64, sh)
        if ev is not None:
            ev[1].record(stream)
        if world > 1:
            gather4()

    steps4 = max(3, min(args.steps, 5))
    el4, km4_local = timed(torch, dist, world, steps4, 1, step4, stream)
    it4_local = int(i4.to(torch.int64).sum().item())
    hist4 = iters_hist(i4.cpu().numpy())
    per4 = per_rank(torch, dist, world, host, dev, [km4_local])
    g4 = time_collective(torch, dist, world, gather4)
    el4, km4, conv4, it4 = reduce_stats(torch, dist, world, host, dev,
                                        [el4, km4_local, int(c4.sum().item()), it4_local], 2)
    del tg4, q4, c4, i4, e4
    if rank == 0:
        ps = el4 / steps4
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        # rank 0's shard, priced like the headline (one GPU's updates over its kernel time)
        rl4, rl4_hbm = roofline("f64", "pair", False, km4_local, it4_local, -(-n // 32), cus * 4,
                                algorithmic_bytes("f64", n), *hbm_profile("f64", n, 0, False))
        rl4["kernel"] = "ikg_pair_batch_kernel (rank 0's shard)"
        extra["c4_strong"] = {
            "workload": f"BASELINE configs[3]: {tot} targets (uniform_targets seed 7) split over {world} rank(s), "
                        "fp64, pair layout; each step the shard solves plus the gather of q, flags and update "
                        "counts to rank 0" + (" (RCCL)" if world > 1 and not host else
                                               " (gloo rehearsal)" if world > 1 else ""),
            "value": conv4 / ps, "unit": "converged solves/s", "problems_per_s": tot / ps,
            "ms_per_step": ps * 1e3, "kernel_ms_max_rank": km4, "scaling": "strong", "n_gpus": world,
            "steps": steps4, "converged_fraction": conv4 / tot,
            "iters_hist": hist4, "iters_hist_is": "rank 0's shard",
            "roofline": rl4, "roofline_hbm": rl4_hbm,
            "ranks": rank_block(per4, world, "nccl" if not host else "gloo", g4,
                                "blocking gather_rows of q, flags and update counts of the whole batch to rank 0, "
                                "wall ms"),
        }
    # ---- C2 with the collision term (the reference's success)
    B = args.batch
    tg = torch.tensor(uniform_targets(B, seed=rank), dtype=torch.float64, device=dev)
    q0 = torch.zeros(15, dtype=torch.float64, device=dev)
    qc = torch.empty((B, 15), dtype=torch.float64, device=dev)
    cc = torch.empty(B, dtype=torch.uint8, device=dev)
    ic = torch.empty(B, dtype=torch.int32, device=dev)
    ec = torch.empty((B, 2), dtype=torch.float64, device=dev)

    def stepc(ev):
        if ev is not None:
            ev[0].record(stream)
        solver.solve_into(tg, q0, qc, cc, ic, ec, _lib.IKG_F64, sh, check_collision=True)
        if ev is not None:
            ev[1].record(stream)

    elc, kmc = timed(torch, dist, world, args.steps, args.warmup, stepc, stream)
    elc, kmc, convc, itc = reduce_stats(torch, dist, world, host, dev,
                                        [elc, kmc, int(cc.sum().item()), int(ic.to(torch.int64).sum().item())], 2)
    if rank == 0:
        ps = elc / args.steps
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        traffic, tsrc = hbm_profile("f64", B, 0, True)
        rl, rl_hbm = roofline("f64", "pair", False, kmc, int(itc), -(-B // 32), cus * 4,
                              algorithmic_bytes("f64", B) + 48 * 8 * 12, traffic, tsrc)
        rl["kernel"], rl["kernel_ms_covers"] = collision_kernels("ikg_pair_batch_kernel", "f64", B)
        rl["work"] += " -- the updates the reference runs; checks are not priced"
        extra["c2_collision"] = {
            "workload": f"BASELINE configs[1] with the reference's success (collision term, "
                        f"inverse_geometry.py:70, :97-98): batch {B} per GPU, fp64",
            "value": convc / ps, "unit": "collision-free converged solves/s", "ms_per_step": ps * 1e3,
            "kernel_ms": kmc, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "converged_fraction": convc / (B * world), "mean_iters": itc / (B * world),
            "iters_hist": iters_hist(ic.cpu().numpy()),
            "roofline": rl, "roofline_hbm": rl_hbm,
        }
    # ---- C2 with random yaw: the "random SE(3)" reading of configs[1] (the
    # reference's "45 deg rotated" case, inverse_geometry_TESTS.py:266)
    yaw = np.pi / 4
    tgy_np = uniform_targets(B, seed=rank, yaw=yaw)
    tgy = torch.tensor(tgy_np, dtype=torch.float64, device=dev)

    def stepy(ev):
        if ev is not None:
            ev[0].record(stream)
        solver.solve_into(tgy, q0, qc, cc, ic, ec, _lib.IKG_F64, sh)
        if ev is not None:
            ev[1].record(stream)

    ely, kmy_local = timed(torch, dist, world, args.steps, args.warmup, stepy, stream)
    ity_local = int(ic.to(torch.int64).sum().item())
    ity_max = int(ic.max().item())
    hist_y = iters_hist(ic.cpu().numpy())
    ely, kmy, convy, ity = reduce_stats(torch, dist, world, host, dev,
                                        [ely, kmy_local, int(cc.sum().item()), ity_local], 2)
    if rank == 0:
        ps = ely / args.steps
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        rl, rl_hbm = roofline("f64", "pair", False, kmy_local, ity_local, -(-B // 32), cus * 4,
                              algorithmic_bytes("f64", B), *hbm_profile("f64", B, 0, False, "yaw"),
                              max_iters=ity_max)
        rl["kernel"] = "ikg_pair_batch_kernel"
        extra["c2_yaw"] = {
            "workload": f"BASELINE configs[1], random SE(3) reading: batch {B} per GPU, fp64, cube yaw ~ "
                        f"U[-pi/4, pi/4] (inverse_geometry_TESTS.py:266 '45 deg rotated'), q0 = 0",
            "value": convy / ps, "unit": "converged solves/s", "ms_per_step": ps * 1e3, "kernel_ms": kmy,
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "converged_fraction": convy / (B * world), "mean_iters": ity / (B * world),
            "iters_hist": hist_y,
            "roofline": rl, "roofline_hbm": rl_hbm,
        }
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(tgy_np, budget_s=6.0, numpy_budget_s=0.0)
            cb.pop("numpy_single_core", None)
            extra["c2_yaw"]["cpu_baseline"] = cb
    return extra


if __name__ == "__main__":
    main()
