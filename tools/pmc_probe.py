"""Run one IK configuration `reps` times (for rocprofv3 --pmc passes).
usage: pmc_probe.py B dtype ppw reps [--save-iters path.npy] [--collision]
                    [--yaw RAD] [--seed N] [--randq0] [--variant V]
--collision: the solve with the collision term (the reference's success).
--yaw: cube yaw ~ U[-RAD, RAD] (bench.py extra.c2_yaw); --seed: the targets'
seed (bench.py c4_strong: 7); --randq0: a random seed row per problem
(workload.random_seeds, seed 1000 -- the multi-start's per-seed problems:
the pair kernel's medium-range instantiation); --variant: ikg_variant;
--multistart S: B targets x S seeds (bench.py --multistart: random_seeds
seed 1000, seed row 0 = q0 = 0), the whole multi-start launch."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "motion-planning-and-control-for-dual-manipulator-robot_amd"))
from ikgrasp.collision import load_nextage_scene  # noqa: E402
from ikgrasp.solver import IKSolver  # noqa: E402
from ikgrasp.workload import uniform_targets  # noqa: E402

B, dtype, ppw, reps = int(sys.argv[1]), sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
col = "--collision" in sys.argv
s = IKSolver(scene=load_nextage_scene() if col else None)
dev = torch.device("cuda", 0)
tdt = torch.float64 if dtype == "f64" else torch.float32
code = 0 if dtype == "f64" else 1
def opt(name, default, conv=float):
    return conv(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


tg = torch.tensor(uniform_targets(B, seed=opt("--seed", 0, int), yaw=opt("--yaw", 0.0)), dtype=tdt, device=dev)
if "--randq0" in sys.argv:
    from ikgrasp.workload import random_seeds  # noqa: E402
    q0 = torch.tensor(random_seeds(s.model, B, seed=1000), dtype=tdt, device=dev)
else:
    q0 = torch.zeros(15, dtype=tdt, device=dev)
qo = torch.empty((B, 15), dtype=tdt, device=dev)
cv = torch.empty(B, dtype=torch.uint8, device=dev)
it = torch.empty(B, dtype=torch.int32, device=dev)
er = torch.empty((B, 2), dtype=tdt, device=dev)
st = torch.cuda.current_stream().cuda_stream
MS = opt("--multistart", 0, int)
if MS:
    from ikgrasp.workload import random_seeds  # noqa: E402
    sd = random_seeds(s.model, MS, seed=1000)
    sd[0] = 0.0
    seeds = torch.tensor(sd, dtype=tdt, device=dev)
    best = torch.empty(B, dtype=torch.int32, device=dev)
for _ in range(reps):
    if MS:
        s.solve_multistart_into(tg, seeds, qo, cv, it, er, best, code, st, check_collision=col,
                                variant=opt("--variant", 0, int))
    else:
        s.solve_into(tg, q0, qo, cv, it, er, code, st, ppw=ppw, check_collision=col, variant=opt("--variant", 0, int))
torch.cuda.synchronize()
print("sum iters", int(it.to(torch.int64).sum()), "converged", int(cv.sum()))
if "--save-iters" in sys.argv:
    import numpy as np
    np.save(sys.argv[sys.argv.index("--save-iters") + 1], it.cpu().numpy())
