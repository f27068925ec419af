"""Kernel time vs dynamic-LDS padding per workgroup (caps workgroups per CU)
and problems per wave; each config in its own process (env var read once)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import os, sys, numpy as np, torch
sys.path.insert(0, os.path.join(%r, "motion-planning-and-control-for-dual-manipulator-robot_amd"))
from ikgrasp.solver import IKSolver
from ikgrasp.workload import uniform_targets
s = IKSolver(); dev = torch.device("cuda", 0)
out = []
for B, dtype in ((4096, "f64"), (4096, "f32"), (65536, "f32"), (65536, "f64")):
    tdt = torch.float64 if dtype == "f64" else torch.float32
    code = 0 if dtype == "f64" else 1
    tg = torch.tensor(uniform_targets(B, seed=0), dtype=tdt, device=dev); q0 = torch.zeros(15, dtype=tdt, device=dev)
    qo = torch.empty((B, 15), dtype=tdt, device=dev); cv = torch.empty(B, dtype=torch.uint8, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev); er = torch.empty((B, 2), dtype=tdt, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    for ppw in (32, 16, 8):
        ts = []
        for r in range(4):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); s.solve_into(tg, q0, qo, cv, it, er, code, st, ppw=ppw); b.record(); torch.cuda.synchronize()
            if r: ts.append(a.elapsed_time(b))
        out.append(f"B={B} {dtype} ppw={ppw}: {np.median(ts):.3f}")
print(" | ".join(out))
''' % ROOT
for pad in (0, 24576, 41984, 54272, 83968):
    env = dict(os.environ, IKG_LDS_PAD=str(pad))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    print(f"pad={pad}: {r.stdout.strip()} {r.stderr.strip()[-300:] if r.returncode else ''}", flush=True)
