# packed fp32 kernel: problems per wave (C3 65536 and C4-share 131072)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pppw; mkdir -p $O
for rep in 1 2; do for v in 64 32 16; do for b in 65536 131072; do
  IKG_PACKED_PPW=$v timeout -k 10 120 python $R/bench.py --no-cpu-baseline --steps 20 --warmup 3 --dtype f32 --batch $b > $O/p${v}_$b.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/p${v}_$b.json')); print('ppw $v B $b', round(d['roofline']['kernel_ms'],4), 'ms')"
done; done; done
