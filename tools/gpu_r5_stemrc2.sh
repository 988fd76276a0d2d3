#!/bin/bash
# stem BN backward reduction with the conv recomputed: stem tests, headline A/B
OUT=${1:-gpurun_out/r5_stemrc2}
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_stem_gpu.py \
  > "$OUT/tests.log" 2>&1 || exit $?
for v in 1 0 1 0; do
  RTSEG_STEM_BN_RECOMPUTE=$v timeout -k 10 300 python3 -u bench.py --no-infer >> "$OUT/bench_r$v.json" 2>> "$OUT/bench.err" || exit $?
done
