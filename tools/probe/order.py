"""Probe: HIP runtime init order between libikgrasp (/opt/rocm runtime) and torch's bundled runtime."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "motion-planning-and-control-for-dual-manipulator-robot_amd"))
import numpy as np
order = sys.argv[1]
if order == "torch_first":
    import torch
    print("torch avail", torch.cuda.is_available())
from ikgrasp.solver import IKSolver
s = IKSolver()
print("fk", s.fk(np.zeros((2, 15)))[0, 0, 9:])
import torch
print("torch avail after", torch.cuda.is_available(), torch.cuda.device_count())
x = torch.ones(4, device="cuda")
print("torch ok", x.sum().item())
