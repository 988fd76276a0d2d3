#!/bin/bash
# One GPU-box session: the whole GPU test tier, KD bench, headline bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/tgpu.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|passed|failed" gpurun_out/tgpu.log | tail -20; exit 1; }
tail -2 gpurun_out/tgpu.log
timeout -k 10 600 python bench.py --steps 10 --warmup 5 --batch 16 --kd --no-infer > gpurun_out/kd.log 2>&1 || { echo KDFAIL; tail -30 gpurun_out/kd.log; exit 1; }
grep metric gpurun_out/kd.log
timeout -k 10 500 python bench.py --steps 10 --warmup 5 > gpurun_out/b32.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/b32.log; exit 1; }
grep metric gpurun_out/b32.log
