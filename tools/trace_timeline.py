"""Kernel timeline of the last bench step from rocprofv3 kernel-trace CSVs
(tools/collision_trace.sh): start/end offsets in us, duration, kernel, for
the last `--last` library kernels (ikg_* and the runtime's fills).
    python tools/trace_timeline.py gpurun_out/coltrace [--last 12]"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default="gpurun_out/coltrace")
    ap.add_argument("--last", type=int, default=12)
    a = ap.parse_args()
    for d in sorted(glob.glob(os.path.join(a.root, "*"))):
        files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        if not files:
            continue
        rows = sorted(csv.DictReader(open(files[0])), key=lambda r: int(r["Start_Timestamp"]))
        rows = [r for r in rows if "ikg" in r["Kernel_Name"] or "fill" in r["Kernel_Name"]][-a.last:]
        t0 = int(rows[0]["Start_Timestamp"])
        print(f"== {d}")
        for r in rows:
            s = (int(r["Start_Timestamp"]) - t0) / 1e3
            e = (int(r["End_Timestamp"]) - t0) / 1e3
            n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ikg::", "")[:70]
            print(f"  {s:9.1f} {e:9.1f} {e - s:8.1f}  {n}")


if __name__ == "__main__":
    main()
