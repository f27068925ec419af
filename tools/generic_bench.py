"""Generic-path benchmark: the synthetic tilted-axis robot
(tests/golden/tilted_dualarm.urdf: runtime axes, placement rotations,
Householder-QR arm solve) against the Nextage specialisation, same batch and
dtype, device-resident inputs, HIP events on the launch stream; each model also
through its run-time specialised kernels (ikg_model_specialize, with the
compile + load time).  One JSON line.
    python tools/generic_bench.py [--batch 4096] [--dtype f64]"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "motion-planning-and-control-for-dual-manipulator-robot_amd"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def time_solver(solver, targets, q0, steps, dtype_code):
    import torch
    B = targets.shape[0]
    q_out = torch.empty((B, solver.nq), dtype=targets.dtype, device="cuda")
    conv = torch.empty(B, dtype=torch.uint8, device="cuda")
    iters = torch.empty(B, dtype=torch.int32, device="cuda")
    err = torch.empty((B, 2), dtype=targets.dtype, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    solver.solve_into(targets, q0, q_out, conv, iters, err, dtype_code, sh)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        solver.solve_into(targets, q0, q_out, conv, iters, err, dtype_code, sh)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    it = int(iters.to(torch.int64).sum().item())
    return {"ms_per_launch": ms, "converged": int(conv.sum().item()), "sum_iters": it,
            "us_per_iteration": ms * 1e3 / (it / B) if it else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from ikgrasp import _lib
    from ikgrasp.model import DualArmModel
    from ikgrasp.solver import IKSolver
    from ikgrasp.workload import uniform_targets
    tdt = torch.float64 if a.dtype == "f64" else torch.float32
    code = _lib.IKG_F64 if a.dtype == "f64" else _lib.IKG_F32
    g = np.load(os.path.join(GOLDEN, "generic_cases.npz"))
    rng = np.random.default_rng(0)
    B = a.batch
    tg = np.repeat(g["targets"][:1], B, axis=0)
    tg[:, 9:] += rng.uniform(-0.05, 0.05, (B, 3))
    tilted = IKSolver(DualArmModel.from_urdf(os.path.join(GOLDEN, "tilted_dualarm.urdf"),
                                             os.path.join(GOLDEN, "tilted_cube.urdf")), specialize=False)
    nextage = IKSolver(specialize=False)
    out = {"bench": "generic path (SURVEY 8f-3)", "batch": B, "dtype": a.dtype}
    out["tilted_generic"] = time_solver(tilted, torch.tensor(tg, dtype=tdt, device="cuda"),
                                        torch.zeros(tilted.nq, dtype=tdt, device="cuda"), a.steps, code)
    out["nextage_specialised"] = time_solver(nextage, torch.tensor(uniform_targets(B, seed=0), dtype=tdt, device="cuda"),
                                             torch.zeros(nextage.nq, dtype=tdt, device="cuda"), a.steps, code)
    import time
    for name, sv in (("tilted", tilted), ("nextage", nextage)):
        t0 = time.time()
        sv.specialize(a.dtype)
        out[f"{name}_specialize_s"] = time.time() - t0
    out["tilted_jit"] = time_solver(tilted, torch.tensor(tg, dtype=tdt, device="cuda"),
                                    torch.zeros(tilted.nq, dtype=tdt, device="cuda"), a.steps, code)
    out["nextage_jit"] = time_solver(nextage, torch.tensor(uniform_targets(B, seed=0), dtype=tdt, device="cuda"),
                                     torch.zeros(nextage.nq, dtype=tdt, device="cuda"), a.steps, code)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
