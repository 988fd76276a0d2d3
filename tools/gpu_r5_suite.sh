#!/bin/bash
# the driver's one-process GPU suite, then a fresh-autotune bench with the per-shape timing table
OUT=${1:-gpurun_out/r5_suite2}
mkdir -p "$OUT"
timeout -k 10 1000 python3 -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1 || exit $?
RTSEG_TUNE_DB=none RTSEG_DECISIONS_OUT="$OUT/decisions.json" timeout -k 10 300 python3 -u bench.py --no-infer \
  > "$OUT/bench_fresh.json" 2> "$OUT/bench_fresh.err"
tools/gpu_pmc.sh gpurun_out/r5_pmc whalo2:128,128,256,128 whalo:64,256,512,64 whalo2:64,256,512,64 \
  hreg2_dg:128,128,256,128 igemm+st:128,128,256,128
