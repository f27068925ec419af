"""Executed FP operations per problem-iteration of the batch kernel, from
rocprofv3 --pmc instruction counters (tools/pmc_flops.sh), for bench.py's
roofline.executed_frac.

A wave-level VALU instruction runs on the wave's 64 lanes; the pair layout
puts 2 lanes on a problem, so one problem-iteration issues (per lane)
2*FMA + MUL + ADD + TRANS FP operations on each of its 2 lanes.  Lanes of
problems that have already stopped are masked off but still occupy the
issue slot, so the counts are divided by the wave-iterations the launch
actually ran: sum over waves of (max updates in the wave + 1 evaluations).

usage: python tools/pmc_flops.py gpurun_out/flops/<dtype>_b<B> B dtype tag"""
import csv
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(d, B, dtype, tag):
    sfx = "F64" if dtype == "f64" else "F32"
    per = {}
    for r in csv.DictReader(open(os.path.join(d, "ops", "run_counter_collection.csv"))):
        if "ikg_pair_batch_kernel" not in r["Kernel_Name"]:
            continue
        per.setdefault(r["Dispatch_Id"], {}).setdefault(r["Counter_Name"], 0.0)
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    it = np.load(os.path.join(d, "iters.npy"))
    ppw = 32
    waves = it.reshape(-1, ppw) if len(it) % ppw == 0 else None
    wave_iters = float((waves.max(axis=1) + 1).sum())
    ops = []
    for c in per.values():
        fp = 2 * c[f"SQ_INSTS_VALU_FMA_{sfx}"] + c[f"SQ_INSTS_VALU_MUL_{sfx}"] + c[f"SQ_INSTS_VALU_ADD_{sfx}"] + \
            c[f"SQ_INSTS_VALU_TRANS_{sfx}"]
        ops.append(fp / wave_iters)
    lane = statistics.median(ops)
    out = {"kernel": "ikg_pair_batch_kernel", "dtype": dtype, "batch": B, "round": tag,
           "fp_ops_per_lane_iter": lane, "fp_ops_per_problem_iter": 2 * lane, "wave_iterations": wave_iters,
           "dispatches": len(ops),
           "note": "rocprofv3 SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS} (FMA = 2 ops) per wave-iteration, x 2 lanes/problem"}
    path = os.path.join(ROOT, "profiles", f"flops_{dtype}_b{B}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, out)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else "r02")
