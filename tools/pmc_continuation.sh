# SQ counters of the collision path's kernels (C2 fp64 --collision, one
# hand-off round so the pair-layout stretch kernel and the continuation both
# run): instructions and wait cycles per wave -> gpurun_out/pmc_cont/
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_cont; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
pass() { name=$1; cnt=$2
  IKG_HANDOFF_ROUNDS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $cnt --output-format csv -d $OUT/$name -o run -- \
    python3 $ROOT/bench.py --collision --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
pass a "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY"
pass b "SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
cd $ROOT
python3 - <<'PY'
import csv, glob, collections
for name in ("a", "b"):
    f = glob.glob(f"gpurun_out/pmc_cont/{name}/**/*counter_collection.csv", recursive=True)
    if not f:
        print("no counters for", name); continue
    rows = list(csv.DictReader(open(f[0])))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ikg::", "")[:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in agg.items():
        if "ikg" not in k and "collide" not in k and "stretch" not in k and "batch" not in k:
            continue
        print(name, k, {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
