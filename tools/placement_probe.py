"""Waves per SIMD of a 1,024-workgroup launch right after (a) a batch solve,
(b) a collision solve (diagnostic for the slow-batch-after-continuation case).
usage: python tools/placement_probe.py"""
import collections
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "motion-planning-and-control-for-dual-manipulator-robot_amd"))
from ikgrasp.collision import load_nextage_scene  # noqa: E402
from ikgrasp.solver import IKSolver  # noqa: E402
from ikgrasp.workload import uniform_targets  # noqa: E402

B = 65536
s = IKSolver(scene=load_nextage_scene())
dev = torch.device("cuda", 0)
tg = torch.tensor(uniform_targets(B, seed=0), dtype=torch.float32, device=dev)
q0 = torch.zeros(15, dtype=torch.float32, device=dev)
qo = torch.empty((B, 15), dtype=torch.float32, device=dev)
cv = torch.empty(B, dtype=torch.uint8, device=dev)
it = torch.empty(B, dtype=torch.int32, device=dev)
er = torch.empty((B, 2), dtype=torch.float32, device=dev)
st = torch.cuda.current_stream().cuda_stream
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "ubench", "bin", "libwhere.so"))
lib.where_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p]
G = 1024
ids = torch.zeros(2 * G, dtype=torch.int32, device=dev)


def placement(tag):
    lib.where_probe(ids.data_ptr(), G, 20000, st)  # 200 us per wave
    torch.cuda.synchronize()
    h = ids.cpu().numpy().astype(np.uint32).reshape(-1, 2)
    simd = collections.Counter()
    for hw, xcc in h:
        simd[(int(xcc) & 0xF, (int(hw) >> 13) & 7, (int(hw) >> 12) & 1, (int(hw) >> 8) & 0xF, (int(hw) >> 4) & 3)] += 1
    hist = collections.Counter(simd.values())
    print(f"{tag}: {len(simd)} SIMDs used; waves-per-SIMD histogram {dict(sorted(hist.items()))}", flush=True)


for k in range(3):
    s.solve_into(tg, q0, qo, cv, it, er, 1, st)
    placement(f"after batch {k}")
for k in range(3):
    s.solve_into(tg, q0, qo, cv, it, er, 1, st, check_collision=True)
    placement(f"after collision solve {k}")
for k in range(2):
    s.solve_into(tg, q0, qo, cv, it, er, 1, st)
    placement(f"after batch again {k}")
