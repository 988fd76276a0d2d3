#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_gpu.py > gpurun_out/t_bn.log 2>&1 || { echo TFAIL; tail -40 gpurun_out/t_bn.log; exit 1; }
tail -1 gpurun_out/t_bn.log
timeout -k 10 400 python bench.py --steps 10 --warmup 5 --no-infer > gpurun_out/b32_bits.log 2>&1 || { echo BFAIL; tail -20 gpurun_out/b32_bits.log; exit 1; }
grep metric gpurun_out/b32_bits.log | cut -c1-220
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_zoo.py -k "cfpnet" > gpurun_out/t_cfp.log 2>&1 || { echo ZFAIL; tail -30 gpurun_out/t_cfp.log; exit 1; }
tail -1 gpurun_out/t_cfp.log
