#!/bin/bash
# One GPU-box session: numerics (conv/BN/dw/misc + zoo), headline bench, DDRNet + BiSeNetV2 profiles.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_conv_gpu.py tests/test_bn_gpu.py tests/test_dwconv_gpu.py tests/test_misc_ops_gpu.py tests/test_ops_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
timeout -k 10 500 python bench.py --steps 10 --warmup 5 > gpurun_out/b32.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/b32.log; exit 1; }
grep metric gpurun_out/b32.log
bash tools/profile_bench.sh gpurun_out/prof_ddr16 --steps 6 --warmup 3 --batch 16 > gpurun_out/prof1.log 2>&1 || { echo PROFFAIL; tail -30 gpurun_out/prof1.log; exit 1; }
head -8 gpurun_out/prof_ddr16/steady.txt
PROF_PER_STEP=5 bash tools/profile_bench.sh gpurun_out/prof_bis16 --steps 6 --warmup 3 --batch 16 --model bisenetv2 > gpurun_out/prof2.log 2>&1 || { echo PROF2FAIL; tail -30 gpurun_out/prof2.log; exit 1; }
head -8 gpurun_out/prof_bis16/steady.txt
