#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > gpurun_out/t_conv.log 2>&1 || { echo TFAIL; tail -40 gpurun_out/t_conv.log; exit 1; }
tail -1 gpurun_out/t_conv.log
timeout -k 10 300 python -u tools/bench_conv.py --batch 1 > gpurun_out/bc1_bm64.log 2>&1 || { echo BCFAIL; tail -20 gpurun_out/bc1_bm64.log; exit 1; }
grep -v amdgpu gpurun_out/bc1_bm64.log
timeout -k 10 300 python -u tools/probe_zoo_err.py bisenetv2 > gpurun_out/pz1.log 2>&1 || { echo PZFAIL; tail -20 gpurun_out/pz1.log; exit 1; }
grep bisenetv2 gpurun_out/pz1.log
MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW=0 timeout -k 10 300 python -u tools/probe_zoo_err.py bisenetv2 > gpurun_out/pz2.log 2>&1 || { echo PZFAIL2; tail -20 gpurun_out/pz2.log; exit 1; }
grep bisenetv2 gpurun_out/pz2.log
