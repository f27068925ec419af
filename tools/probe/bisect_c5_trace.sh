# kernel durations of the C5 share fp32 solve, old tree vs HEAD
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; V=$R/motion-planning-and-control-for-dual-manipulator-robot_amd/ikgrasp/_native/var/bis; O=$R/gpurun_out/bist; mkdir -p $O
for c in 5df86e0 HEAD; do
  d=$V/$c; [ $c = HEAD ] && d=$R
  va=""; [ $c != 5df86e0 ] && va="--variant 1"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$c -o run -- python3 $d/bench.py --no-cpu-baseline --steps 5 --warmup 1 --dtype f32 --batch 512 --multistart 256 $va > $O/$c.json 2>/dev/null || exit 1
done
