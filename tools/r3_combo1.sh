#!/bin/bash
tools/r3_bisect.sh && tools/r3_col_ab.sh && \
  timeout -k 10 600 python -u -m pytest -s -q --timeout 300 --timeout-method thread tests/test_gpu_collision.py tests/test_gpu_parity.py -k "fp32 or b65536" > gpurun_out/colab/pytest_gates.log 2>&1; echo "pytest rc=$?"; grep -E "flag flips|success flags differ|passed|failed" gpurun_out/colab/pytest_gates.log | head -20
