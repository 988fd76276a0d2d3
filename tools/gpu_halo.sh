#!/bin/bash
# halo conv: numerics tests, then the per-shape timing table vs MIOpen and the gather kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/halo_pytest.log 2>&1 || { echo TFAIL; tail -40 gpurun_out/halo_pytest.log; exit 1; }
tail -3 gpurun_out/halo_pytest.log
timeout -k 10 400 python -u tools/bench_conv.py --only fwd,dgrad --shapes 0,2,4,6 --iters 30 > gpurun_out/halo_bench.txt 2>&1 || { echo BFAIL; tail -20 gpurun_out/halo_bench.txt; exit 1; }
cat gpurun_out/halo_bench.txt
