# C5 share (256 seeds x 512 targets, fp32): pair vs packed layout
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/c5v; mkdir -p $O
for rep in 1 2; do for v in 0 1 2; do
  timeout -k 10 120 python $R/bench.py --no-cpu-baseline --steps 10 --warmup 2 --dtype f32 --batch 512 --multistart 256 --variant $v > $O/v${v}.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/v${v}.json')); print('variant $v', round(d['ms_per_step'],3), 'ms', d['roofline'].get('kernel'))"
done; done
