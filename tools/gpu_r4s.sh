# Trajectory-scan statistics at C3 fp32 with the collision term (IKG_CPROF build,
# tools/cprof.sh): trajectory windows (default) and records-in-batch (pair, raised budget)
O=gpurun_out/${SCANTAG:-r4s}; mkdir -p $O
export IKGRASP_LIB=$(pwd)/ab_libs/diag/libikgrasp_cprof.so  # abl/ is not uploaded
timeout -k 10 120 python tools/scan_prof.py 65536 f32 > $O/c3_traj.json 2>>$O/err || exit 1
IKG_REC_BUDGET_MB=8192 IKG_REC_PREFER_PAIR=1 timeout -k 10 120 python tools/scan_prof.py 65536 f32 > $O/c3_rec.json 2>>$O/err || exit 1
timeout -k 10 120 python tools/scan_prof.py 4096 f64 > $O/c2_rec.json 2>>$O/err || exit 1
cat $O/*.json
