O=gpurun_out/scanprof; mkdir -p $O
for w in 128 1001; do
  IKG_TRAJ_WINDOW=$w timeout -k 10 120 python tools/scan_prof.py 4096 f64 > $O/c2_w$w.json 2>>$O/err || exit 1
  IKG_TRAJ_WINDOW=$w timeout -k 10 120 python tools/scan_prof.py 65536 f32 > $O/c3_w$w.json 2>>$O/err || exit 1
done
cat $O/*.json
