# A/B of collision-continuation builds (var/lib_*.so): kernel times of the --collision benches
ROOT=$(pwd); O=$ROOT/gpurun_out/colab; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
for lib in $ROOT/motion-planning-and-control-for-dual-manipulator-robot_amd/ikgrasp/_native/var/lib_*.so; do
  n=$(basename $lib .so)
  for cfg in "c2 --collision" "c3 --collision --dtype f32 --batch 65536"; do set -- $cfg; t=$1; shift
    IKGRASP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${n}_$t -o run -- \
      python3 $ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@" > $O/${n}_$t.json 2>/dev/null || exit 1
    python3 - $O/${n}_$t <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "ikg_" in r["Name"]]
solves = max(int(r["Calls"]) for r in rows if "batch_kernel" in r["Name"])
tot = 0.0
for r in rows:  # per solve: a kernel launched k times per solve counts k launches
    ms = float(r["TotalDurationNs"]) / 1e6 / solves
    tot += ms
    print(sys.argv[1].split("/")[-1], r["Name"][:40], round(ms, 3), "ms/solve", int(r["Calls"]) // solves, "launches")
print(sys.argv[1].split("/")[-1], "TOTAL", round(tot, 3), "ms/solve")
PY
  done
done
