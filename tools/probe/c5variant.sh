# C5 share (256 seeds x 512 targets, fp32): AUTO / pair / packed layouts (kernel names from rocprof)
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/c5v; mkdir -p $O
for v in 0 1 2; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v$v -o run -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 2 --dtype f32 --batch 512 --multistart 256 --variant $v > $O/v${v}.json 2>/dev/null || exit 1
  python3 -c "
import json,csv,glob
d=json.load(open('$O/v${v}.json')); f=glob.glob('$O/v$v/**/*kernel_stats.csv',recursive=True)[0]
k=[r for r in csv.DictReader(open(f)) if 'batch_kernel' in r['Name']][0]
print('variant $v', round(d['ms_per_step'],3), 'ms', k['Name'][:40], round(float(k['AverageNs'])/1e3,1), 'us')"
done
