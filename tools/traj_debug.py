"""Trajectory continuation consistency probe: repeated solves and the three
schedules on the graph test's batch (B = 1024, seeds 3 and 4)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "motion-planning-and-control-for-dual-manipulator-robot_amd"))
import numpy as np
from ikgrasp.collision import load_nextage_scene
from ikgrasp.solver import IKSolver
from ikgrasp.workload import uniform_targets
s = IKSolver(device=0, scene=load_nextage_scene())
for seed in (3, 4):
    tg = uniform_targets(1024, seed=seed)
    res = {}
    for name, env in [("def", {}), ("def2", {}), ("def3", {}), ("pre", {"IKG_TRAJ_PRESCREEN": "1"}),
                      ("sep", {"IKG_TRAJ_FUSE": "0"}), ("old", {"IKG_CONT_TRAJ": "0"})]:
        for k in ("IKG_TRAJ_PRESCREEN", "IKG_TRAJ_FUSE", "IKG_CONT_TRAJ"):
            os.environ.pop(k, None)
        os.environ.update(env)
        r = s.solve(tg, np.zeros(15), check_collision=True)
        res[name] = r
    base = res["old"]
    for name, r in res.items():
        dc = np.flatnonzero(r.converged != base.converged)
        di = np.flatnonzero(r.iters != base.iters)
        print(seed, name, "conv", int(r.converged.sum()), "flag diffs", dc[:8].tolist(), len(dc), "iter diffs", len(di),
              "maxdq", float(np.abs(r.q - base.q).max()))
    free = s.solve(tg, np.zeros(15))
    cv = free.converged.astype(bool)
    col = s.collision(free.q[cv], tg[cv])
    print(seed, "first-check colliding", int(col.sum()), "of", int(cv.sum()))
