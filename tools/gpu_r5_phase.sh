#!/bin/bash
# twin-node phase-(0,0) shortcut dgrad: kernel + block tests, headline A/B
OUT=${1:-gpurun_out/r5_phase}
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_igemm_gpu.py \
  tests/test_conv_gemm.py tests/test_conv_stem_gpu.py > "$OUT/tests.log" 2>&1 || exit $?
for v in 1 0 1; do
  RTSEG_TWIN_PHASE=$v timeout -k 10 300 python3 -u bench.py --no-infer >> "$OUT/bench_p$v.json" 2>> "$OUT/bench.err" || exit $?
done
