#!/bin/bash
# 4-channel stem staging: stem tests, stem PMC, headline bench
OUT=${1:-gpurun_out/r5_stem4}
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_stem_gpu.py \
  > "$OUT/tests.log" 2>&1 || exit $?
tools/gpu_r5_stempmc.sh > "$OUT/pmc.log" 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-infer >> "$OUT/bench.json" 2>> "$OUT/bench.err" || exit $?
done
