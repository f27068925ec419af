#!/bin/bash
# Jacobi-call A/B, then the GPU suite (and a poisoned collision/graph pass) on the in-tree library.
ROOT=$(pwd); O=$ROOT/gpurun_out/combo2; mkdir -p $O
tools/r3_ab13.sh || exit 3
timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -1 $O/pytest.log
IKG_POISON=1 timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_collision.py tests/test_gpu_graph.py > $O/pytest_poison.log 2>&1; echo "poison rc=$?"; tail -1 $O/pytest_poison.log
