# A/B of the controller kernel: the built library against
# ikgrasp/_native/var/lib_ctl_old.so, interleaved, per output set -> gpurun_out/ctlab/
set -o pipefail
mkdir -p gpurun_out/ctlab
N=motion-planning-and-control-for-dual-manipulator-robot_amd/ikgrasp/_native
for rep in 1 2; do
  for o in ${SETS:-J pv err task jac all}; do
    for lib in new old; do
      L=$N/libikgrasp.so; [ $lib = old ] && L=$N/var/lib_ctl_old.so
      IKGRASP_LIB=$L timeout -k 10 120 python tools/control_bench.py --outputs $o --no-cpu > gpurun_out/ctlab/${o}_${lib}_$rep.json || exit $?
    done
  done
done
SETS="${SETS:-J pv err task jac all}" python3 - <<'PY'
import json
import os
for o in os.environ.get("SETS", "J pv err task jac all").split():
    row = []
    for lib in ("new", "old"):
        ms = [json.load(open(f"gpurun_out/ctlab/{o}_{lib}_{r}.json"))["ms_per_launch"] for r in (1, 2)]
        row.append(f"{lib} {min(ms):.3f}/{max(ms):.3f}")
    print(o, *row)
PY
