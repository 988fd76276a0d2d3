#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_conv_halo_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ig2_pytest.log 2>&1 || { echo TFAIL; tail -40 gpurun_out/ig2_pytest.log; exit 1; }
tail -2 gpurun_out/ig2_pytest.log
timeout -k 10 400 python -u tools/bench_conv.py --only fwd,dgrad --iters 20 > gpurun_out/ig2_bench.txt 2>&1 || { tail -20 gpurun_out/ig2_bench.txt; exit 1; }
cat gpurun_out/ig2_bench.txt
