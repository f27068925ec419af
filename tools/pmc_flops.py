"""Executed FP operations per problem-iteration of a batch kernel, from
rocprofv3 --pmc instruction counters (tools/pmc_flops.sh), for bench.py's
roofline.executed.

Pair layout (ikg_pair_batch_kernel): 2 lanes per problem, 32 problems per
wave; one problem-iteration issues (per lane) 2*FMA + MUL + ADD + TRANS FP
operations on each of its 2 lanes.  Packed layout (ikg_packed_batch_kernel,
fp32): one lane per problem, 64 problems per wave, both arms in 2-vectors;
SQ_INSTS_VALU_*_F32 count a v_pk_* instruction once, so its second half is
counted from the packed-instruction counter (SQ_INSTS_VALU_PK_* is not
collected on gfx950 here: the figure is a lower bound and says so).
Lanes of problems that have already stopped are masked off but still occupy
the issue slot, so the counts are divided by the wave-iterations the launch
actually ran: sum over waves of (max updates in the wave + 1 evaluations).

usage: python tools/pmc_flops.py gpurun_out/flops/<dtype>_b<B> B dtype tag [--med]
--med: the medium-range (per-problem seeds, multi-start) instantiation ->
profiles/flops_<layout>_<dtype>_med.json (bench.py flops_profile)."""
import csv
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"ikg_pair_batch_kernel": ("pair", 32, 2), "ikg_packed_batch_kernel": ("packed", 64, 1)}


def main(d, B, dtype, tag):
    sfx = "F64" if dtype == "f64" else "F32"
    per, kname = {}, None
    for r in csv.DictReader(open(os.path.join(d, "ops", "run_counter_collection.csv"))):
        k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
        if k is None:
            continue
        kname = k
        per.setdefault(r["Dispatch_Id"], {}).setdefault(r["Counter_Name"], 0.0)
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    short, ppw, lanes = KERNELS[kname]
    it = np.load(os.path.join(d, "iters.npy"))
    pad = (-len(it)) % ppw
    waves = np.concatenate([it, np.full(pad, -1)]).reshape(-1, ppw)
    wave_iters = float((waves.max(axis=1) + 1).sum())
    ops = []
    for c in per.values():
        fp = 2 * c[f"SQ_INSTS_VALU_FMA_{sfx}"] + c[f"SQ_INSTS_VALU_MUL_{sfx}"] + c[f"SQ_INSTS_VALU_ADD_{sfx}"] + \
            c[f"SQ_INSTS_VALU_TRANS_{sfx}"]
        ops.append(fp / wave_iters)
    lane = statistics.median(ops)
    out = {"kernel": kname, "dtype": dtype, "batch": B, "round": tag, "problems_per_wave": ppw,
           "fp_ops_per_lane_iter": lane, "fp_ops_per_problem_iter": lanes * lane, "wave_iterations": wave_iters,
           "dispatches": len(ops),
           "note": f"rocprofv3 SQ_INSTS_VALU_{{FMA,MUL,ADD,TRANS}}_{sfx} (FMA = 2 ops) per wave-iteration, "
                   f"x {lanes} lane(s)/problem" +
                   ("; v_pk_* instructions counted once (lower bound: each carries both arms)"
                    if short == "packed" else "")}
    med = "--med" in sys.argv
    if med:
        out["instantiation"] = "medium-range trig rule (per-problem q0 rows / multi-start seeds)"
    path = os.path.join(ROOT, "profiles", f"flops_{short}_{dtype}_med.json" if med else
                        f"flops_{short}_{dtype}.json" if short == "packed" else f"flops_{dtype}_b{B}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, out)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(args[0], int(args[1]), args[2], args[3] if len(args) > 3 else "r03")
