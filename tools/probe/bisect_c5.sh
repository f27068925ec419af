# fp32 pair-layout timing across older trees (var/bis/<commit>) and HEAD: C5 share and C4 share
R=$GRAFT_REPO_ROOT; V=$R/motion-planning-and-control-for-dual-manipulator-robot_amd/ikgrasp/_native/var/bis; O=$R/gpurun_out/bis; mkdir -p $O
for c in 5df86e0 7cb97f0 HEAD; do
  d=$V/$c; [ $c = HEAD ] && d=$R
  for cfg in "c5 --batch 512 --multistart 256" "c4 --batch 131072" "c2 --batch 4096"; do set -- $cfg; t=$1; shift
    va=""; [ $c != 5df86e0 ] && va="--variant 1"
    (cd $d && timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --dtype f32 $va "$@" > $O/${c}_$t.json 2>$O/${c}_$t.err) || { echo "$c $t failed"; tail -3 $O/${c}_$t.err; continue; }
    python -c "import json; d=json.load(open('$O/${c}_$t.json')); print('$c $t', round(d['ms_per_step'],3), 'ms', round(d['value']))"
  done
done
