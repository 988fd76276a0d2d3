#!/bin/bash
# One GPU-box session: kernel numerics tests, then the headline bench (batch 8 and 16).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_dwconv_gpu.py tests/test_misc_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 400 python bench.py --steps 10 --warmup 5 > gpurun_out/b8.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/b8.log; exit 1; }
grep metric gpurun_out/b8.log
timeout -k 10 400 python bench.py --steps 10 --warmup 5 --batch 16 --no-infer > gpurun_out/b16.log 2>&1 || { echo BENCH16FAIL; tail -30 gpurun_out/b16.log; exit 1; }
grep metric gpurun_out/b16.log
