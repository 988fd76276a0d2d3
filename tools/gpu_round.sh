#!/bin/bash
# One GPU-box session: benches (filling the in-tree MIOpen find db), rocprofv3 profiles.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --steps 10 --warmup 5 --batch 32 --no-infer > gpurun_out/b32.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/b32.log; exit 1; }
grep metric gpurun_out/b32.log
timeout -k 10 400 python bench.py --steps 10 --warmup 5 --batch 16 --model bisenetv2 --no-infer > gpurun_out/bis.log 2>&1 || { echo BISFAIL; tail -30 gpurun_out/bis.log; exit 1; }
grep metric gpurun_out/bis.log
timeout -k 10 500 python bench.py --steps 10 --warmup 5 --batch 16 > gpurun_out/b16.log 2>&1 || { echo B16FAIL; tail -30 gpurun_out/b16.log; exit 1; }
grep metric gpurun_out/b16.log
du -sh miopen_db; ls miopen_db | head; cp -r miopen_db gpurun_out/miopen_db_new
