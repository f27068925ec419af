"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/pmc_run.sh) into
profiles/pmc_<dtype>_b<B>.json, read by bench.py for roofline.traffic.

FETCH_SIZE/WRITE_SIZE are KiB per dispatch (TCC_EA0_RDREQ/WRREQ x 64 B).  Per
MI355X_MICROARCH.md §HBM, gfx950's FETCH_SIZE reports half the bytes of a wide
coalesced read, so it is doubled; WRITE_SIZE is taken as is."""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(d, counter):
    vals = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if ("ikg_pair_batch_kernel" in r["Kernel_Name"] or "ikg_packed_batch_kernel" in r["Kernel_Name"]) \
                and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def per_solve(d, counter, solves):
    """Collision solves launch several kernels (batch kernel, pre-screen, scan,
    compaction): every ikg_* dispatch of the run, summed, over the number of
    identical solves the probe ran."""
    tot = 0.0
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Kernel_Name"].startswith("ikg_") or " ikg_" in r["Kernel_Name"] or "ikg::" in r["Kernel_Name"]:
            if r["Counter_Name"] == counter:
                tot += float(r["Counter_Value"])
    return tot / solves


def main_collision(pmc_dir, dtype, B, tag, solves, S=0, col=True):
    # every ikg_* dispatch of a run over its solves: a collision solve, or
    # (S > 0) a multi-start launch with or without the collision term
    x = (f"_s{S}" if S else "") + ("_col" if col else "")
    fetch = per_solve(os.path.join(pmc_dir, f"fetch_b{B}_{dtype}{x}"), "FETCH_SIZE", solves)
    write = per_solve(os.path.join(pmc_dir, f"write_b{B}_{dtype}{x}"), "WRITE_SIZE", solves)
    what = (f"multi-start launch ({S} seeds x {B} targets): every ikg_* kernel of one ikg_solve_multistart"
            if S else "collision solve: every ikg_* kernel of one ikg_solve_batch") + \
        (" with check_collision" if col else "")
    out = {"kernel": what,
           "dtype": dtype, "batch": B, "round": tag, "solves": solves,
           "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write, "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
           "note": "2 x FETCH_SIZE (gfx950 wide-read correction) + WRITE_SIZE, KiB -> bytes; all dispatches of "
                   "the run over the number of identical solves"}
    if S:
        out["seeds_per_target"] = S
    path = os.path.join(ROOT, "profiles", f"pmc_{dtype}_b{B}{x}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, out)


def main(pmc_dir, dtype, B, tag, sfx=""):
    x = f"_{sfx}" if sfx else ""
    fetch = statistics.median(per_dispatch(os.path.join(pmc_dir, f"fetch_b{B}_{dtype}{x}"), "FETCH_SIZE"))
    write = statistics.median(per_dispatch(os.path.join(pmc_dir, f"write_b{B}_{dtype}{x}"), "WRITE_SIZE"))
    out = {
        "kernel": "ikg_packed_batch_kernel" if (dtype == "f32" and B >= 65536) else "ikg_pair_batch_kernel",
        "dtype": dtype, "batch": B, "round": tag,
        "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
        "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
        "note": "2 x FETCH_SIZE (gfx950 wide-read correction) + WRITE_SIZE, KiB -> bytes; median over dispatches",
    }
    if sfx:
        out["workload"] = sfx
    path = os.path.join(ROOT, "profiles", f"pmc_{dtype}_b{B}{x}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, out)


if __name__ == "__main__":
    # pmc_summary.py DIR dtype B tag --multistart S SOLVES [--collision]
    if "--multistart" in sys.argv:
        i = sys.argv.index("--multistart")
        main_collision(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4], int(sys.argv[i + 2]),
                       S=int(sys.argv[i + 1]), col="--collision" in sys.argv)
        sys.exit(0)
    if "--collision" in sys.argv:
        main_collision(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4], int(sys.argv[6]))
        sys.exit(0)
    sfx = next((a[6:] for a in sys.argv if a.startswith("--sfx=")), "")
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(args[0], args[1], int(args[2]), args[3] if len(args) > 3 else "r01", sfx)
