#!/bin/bash
# masked residual-gradient hand-off: dgrad kernel tests, handoff equality, A/B bench; igemm cfg sweep
OUT=${1:-gpurun_out/r5_masked}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_igemm_gpu.py \
  tests/test_conv_wres_gpu.py tests/test_conv_halo_gpu.py tests/test_conv_gemm.py tests/test_bn_gpu.py \
  > "$OUT/tests.log" 2>&1 || exit $?
for v in 1 0 1; do
  RTSEG_MASKED_HANDOFF=$v timeout -k 10 300 python3 -u bench.py --no-infer >> "$OUT/bench_m$v.json" 2>> "$OUT/bench.err" || exit $?
done
timeout -k 10 500 python3 -u tools/bench_igemm_cfg.py > "$OUT/igemm_cfg.txt" 2>&1
