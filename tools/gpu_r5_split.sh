#!/bin/bash
# BN finalize row-split pre-pass: numerics (BN, SyncBN, zoo DDRNet) then the headline A/B and a profile
OUT=${1:-gpurun_out/r5_split}
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_gpu.py \
  tests/test_syncbn_gpu.py tests/test_conv_gemm.py tests/test_conv_stem_gpu.py > "$OUT/tests.log" 2>&1 || exit $?
for v in 1 0 1; do
  RTSEG_BN_SPLIT=$v timeout -k 10 300 python3 -u bench.py --no-infer >> "$OUT/bench_split$v.json" 2>> "$OUT/bench.err" || exit $?
done
tools/profile_bench.sh "$OUT/prof" --steps 6 --warmup 3
