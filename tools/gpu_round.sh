#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_misc_ops_gpu.py tests/test_detail_loss_gpu.py > gpurun_out/t_col.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_col.log; exit 1; }
tail -2 gpurun_out/t_col.log
