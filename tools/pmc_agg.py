"""Aggregate rocprofv3 counter CSVs of tools/pmc_mix.sh for one kernel name fragment.
usage: python tools/pmc_agg.py gpurun_out/pmc_TAG kernel_fragment"""
import collections
import csv
import glob
import sys

d, frag = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in sorted(glob.glob(d + "/p*/run_counter_collection.csv")):
    for x in csv.DictReader(open(f)):
        if frag in x["Kernel_Name"]:
            agg[x["Counter_Name"]] += float(x["Counter_Value"])
            disp[x["Counter_Name"]].add(x["Dispatch_Id"])
for k in sorted(agg):
    print(f"{k:32s} {agg[k]:16.0f}  per-dispatch {agg[k] / max(1, len(disp[k])):14.0f}")
