#!/usr/bin/env python3
"""SQ occupancy / issue counters of one kernel from rocprofv3 --pmc passes
(tools/pmc_pass.sh with SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY),
per dispatch, with the derived VALU-pipe utilisation.  SQ_WAVE_CYCLES,
SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md, PMC
table); WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES.

usage: tools/sq_summary.py OUT.json KERNEL_SUBSTR label=DIR [label=DIR ...]
"""
import collections
import csv
import json
import sys


def one(d, ksub):
    acc = collections.defaultdict(float)
    ndisp = set()
    dur = []
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if ksub not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Dispatch_Id"] not in ndisp:
            ndisp.add(r["Dispatch_Id"])
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    n = len(ndisp)
    c = {k: v / n for k, v in acc.items()}
    wc = c["SQ_WAVE_CYCLES"]
    out = dict(dispatches=n, counters_per_dispatch={k: round(v) for k, v in c.items()},
               kernel_ms_under_counters=round(1e3 * sum(dur) / n, 4),
               wait_inst_any_frac_of_wave_cycles=round(c["SQ_WAIT_INST_ANY"] / wc, 4),
               wait_any_frac_of_wave_cycles=round(c["SQ_WAIT_ANY"] / wc, 4),
               active_inst_valu_frac_of_wave_cycles=round(c["SQ_ACTIVE_INST_VALU"] / wc, 4))
    return out


def main():
    out_path, ksub = sys.argv[1], sys.argv[2]
    res = dict(kernel_substr=ksub, units="SQ_WAVE_CYCLES / WAIT_* / ACTIVE_INST_* in quad-cycles", runs={})
    for a in sys.argv[3:]:
        lab, d = a.split("=", 1)
        res["runs"][lab] = one(d, ksub)
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
