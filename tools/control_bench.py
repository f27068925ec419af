"""Controller-row benchmark: ikg_frame_kinematics_batch over a
batch of robot states resident in HBM, timed with HIP events on the launch
stream; HBM roofline from the algorithmic bytes; the numpy control oracle
timed beside it on one host core.  One JSON line.

    python tools/control_bench.py [--batch 1048576] [--dtype f64] [--outputs all|task|jac] [--rf 2]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "motion-planning-and-control-for-dual-manipulator-robot_amd"))

SETS = {
    "all": ("placement", "velocity", "J", "dJ", "dJv", "err", "derr"),
    "task": ("placement", "velocity", "J", "dJv", "err", "derr"),  # control.task_space_terms
    "jac": ("J", "dJ"),
    # breakdown of the task set
    "J": ("J",),
    "pv": ("placement", "velocity"),
    "pvj": ("placement", "velocity", "J", "dJv"),
    "err": ("err", "derr"),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--outputs", default="all", choices=sorted(SETS))
    ap.add_argument("--rf", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    import torch
    from ikgrasp import _lib
    from ikgrasp.solver import IKSolver

    s = IKSolver(device=0)
    nq = s.nq
    tdt = torch.float64 if a.dtype == "f64" else torch.float32
    esz = 8 if a.dtype == "f64" else 4
    B = a.batch
    g = torch.Generator(device="cuda").manual_seed(0)
    lo = torch.tensor(s.model.lower, device="cuda", dtype=tdt)
    hi = torch.tensor(s.model.upper, device="cuda", dtype=tdt)
    q = lo + (hi - lo) * torch.rand(B, nq, generator=g, device="cuda", dtype=tdt)
    v = torch.randn(B, nq, generator=g, device="cuda", dtype=tdt)
    qd = q + 0.05 * torch.randn(B, nq, generator=g, device="cuda", dtype=tdt)
    vd = v + 0.1 * torch.randn(B, nq, generator=g, device="cuda", dtype=tdt)
    outs = SETS[a.outputs]
    shapes = {"placement": 24, "velocity": 12, "J": 12 * nq, "dJ": 12 * nq, "dJv": 12, "err": 12, "derr": 12}
    res = {k: torch.empty(B, shapes[k], device="cuda", dtype=tdt) for k in outs}
    des = "err" in outs or "derr" in outs
    fo = _lib.FrameKinOut(*[res[k].data_ptr() if k in res else None for k in s.FRAME_KIN_OUTPUTS])
    stream = torch.cuda.current_stream().cuda_stream
    code = _lib.IKG_F64 if a.dtype == "f64" else _lib.IKG_F32

    def launch():
        _lib.check(s.lib.ikg_frame_kinematics_batch(
            s._h, 0, code, q.data_ptr(), v.data_ptr(), qd.data_ptr() if des else None,
            vd.data_ptr() if des else None, B, a.rf, C.byref(fo), C.c_void_p(stream), 0))

    for _ in range(a.warmup):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    in_bytes = (4 if des else 2) * nq * esz
    out_bytes = sum(shapes[k] for k in outs) * esz
    per_state = in_bytes + out_bytes
    gbs = per_state * B / (ms * 1e-3) / 1e9
    traffic = None  # measured HBM bytes per launch (tools/control_pmc.sh), for this exact configuration
    pmc = os.path.join(ROOT, "profiles", "r01", "control", f"pmc_{a.outputs}_{a.dtype}_b{B}.json")
    if a.rf == 2 and os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
    line = {
        "bench": "controller kinematics (SURVEY 8f-4): ikg_frame_kinematics_batch",
        "batch": B, "dtype": a.dtype, "rf": a.rf, "outputs": list(outs),
        "ms_per_launch": ms, "states_per_s": B / (ms * 1e-3),
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": gbs / HBM_PEAK_GBS, "traffic": traffic, "algorithmic_bytes_per_state": per_state,
                     "kernel": "ikg_frame_kin_kernel"},
    }
    if not a.no_cpu:
        from oracle import control_oracle as co
        qn, vn = q[:64].double().cpu().numpy(), v[:64].double().cpu().numpy()
        qdn, vdn = qd[:64].double().cpu().numpy(), vd[:64].double().cpu().numpy()
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 3.0:
            i = n % 64
            co.frame_kinematics(qn[i], vn[i], a.rf, qdn[i] if des else None, vdn[i] if des else None)
            n += 1
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": n / dt, "unit": "states/s", "cores": 1, "kind": "port",
                                "sample": f"{n} states through oracle/control_oracle.py (numpy spatial algebra, "
                                          f"Pinocchio's formulation), {dt:.1f} s"}
    print(json.dumps(line))
    s.close()


if __name__ == "__main__":
    main()
