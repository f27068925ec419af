# interleaved bench.py timing of var/lib_*.so builds (headline configs)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/abb; mkdir -p $O
for rep in 1 2; do
for lib in $R/motion-planning-and-control-for-dual-manipulator-robot_amd/ikgrasp/_native/var/lib_*.so; do n=$(basename $lib .so)
  for cfg in "c2 --batch 4096" "c3 --dtype f32 --batch 65536" "c3d --dtype f64 --batch 65536"; do set -- $cfg; t=$1; shift
    IKGRASP_LIB=$lib timeout -k 10 120 python $R/bench.py --no-cpu-baseline --steps 20 --warmup 3 "$@" > $O/${n}_${t}_$rep.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/${n}_${t}_$rep.json')); print('$n $t $rep', round(d['ms_per_step'],4), 'ms', round(d['roofline']['kernel_ms'],4) if 'kernel_ms' in d['roofline'] else '')"
  done
done; done
