# Interleaved A/B of the built library against ikgrasp/_native/var/*.so on the
# fp32 configurations (C3 B=65,536 from q=0, 131,072, random seeds), 30 rounds.
set -o pipefail
N=motion-planning-and-control-for-dual-manipulator-robot_amd/ikgrasp/_native
L="$N/libikgrasp.so $N/var/*.so"
export ABL_ROUNDS=${ABL_ROUNDS:-30}
timeout -k 10 300 python tools/ablate.py 65536 f32 "$L" 2>&1 | grep "B=" || exit $?
timeout -k 10 300 python tools/ablate.py 131072 f32 "$L" 2>&1 | grep "B=" || exit $?
ABL_RANDQ0=1 timeout -k 10 300 python tools/ablate.py 65536 f32 "$L" 2>&1 | grep "B=" || exit $?
