#!/bin/bash
# conv numerics tests, then the default bench (DDRNet-23 b32) with the per-shape kernel decisions
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_conv_halo_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q_pytest.log 2>&1 || { echo TFAIL; tail -40 gpurun_out/q_pytest.log; exit 1; }
tail -2 gpurun_out/q_pytest.log
RTSEG_DECISIONS_OUT=gpurun_out/q_decisions.txt timeout -k 10 400 python -u bench.py > gpurun_out/q_bench.log 2>&1 || { echo BFAIL; tail -20 gpurun_out/q_bench.log; exit 1; }
tail -1 gpurun_out/q_bench.log
