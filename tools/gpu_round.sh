#!/bin/bash
# One GPU-box session: zoo error probe, numerics (conv/BN/zoo), headline bench, DDRNet profile.
set -o pipefail
mkdir -p gpurun_out


timeout -k 10 900 python -u -m pytest tests/test_conv_gpu.py tests/test_bn_gpu.py tests/test_zoo.py -m gpu -q --timeout 120 --timeout-method thread -k "dfanet or conv or bn" > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
timeout -k 10 500 python bench.py --steps 10 --warmup 5 > gpurun_out/b32.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/b32.log; exit 1; }
grep metric gpurun_out/b32.log
bash tools/profile_bench.sh gpurun_out/prof_ddr16 --steps 6 --warmup 3 --batch 16 > gpurun_out/prof1.log 2>&1 || { echo PROFFAIL; tail -30 gpurun_out/prof1.log; exit 1; }
head -30 gpurun_out/prof_ddr16/steady.txt
