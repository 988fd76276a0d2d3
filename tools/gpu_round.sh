#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_misc_ops_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
timeout -k 10 500 python bench.py --steps 10 --warmup 5 --no-infer > gpurun_out/b32.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/b32.log; exit 1; }
grep metric gpurun_out/b32.log
bash tools/profile_bench.sh gpurun_out/prof_ddr16 --steps 6 --warmup 3 --batch 16 > gpurun_out/prof1.log 2>&1 || { echo PROFFAIL; tail -30 gpurun_out/prof1.log; exit 1; }
head -8 gpurun_out/prof_ddr16/steady.txt; grep -n "fused_opt\|ema_lerp\|multi_tensor" gpurun_out/prof_ddr16/steady.txt | cut -c1-120
