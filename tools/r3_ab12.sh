#!/bin/bash
ROOT=$(pwd); O=$ROOT/gpurun_out/ab12; mkdir -p $O
L="$ROOT/ab_libs/*.so"
ABL_COLLISION=1 ABL_EPS=1e-3 ABL_ROUNDS=12 timeout -k 10 300 python tools/ablate.py 4096 f64 "$L" > $O/c2col_f64.txt 2>&1 || exit 3
ABL_COLLISION=1 ABL_EPS=1e-3 ABL_ROUNDS=6 timeout -k 10 300 python tools/ablate.py 65536 f32 "$L" > $O/c3col_f32.txt 2>&1 || exit 3
grep -H median $O/*.txt
timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 $O/pytest.log; IKG_POISON=1 timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_collision.py tests/test_gpu_graph.py > $O/pytest_poison.log 2>&1; echo "poison rc=$?"; tail -1 $O/pytest_poison.log
