#!/bin/bash
ROOT=$(pwd); O=$ROOT/gpurun_out/s2d; mkdir -p $O
IKG_REPORT_DIR=$O/reports timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_sharded.py -v -s --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|c5_share|c3_vs" $O/pytest.log | tail -20
exit $rc
