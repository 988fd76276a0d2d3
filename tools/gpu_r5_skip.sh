#!/bin/bash
# skip-gradient hand-off (bilateral fusion): tests, headline A/B, op probe
OUT=${1:-gpurun_out/r5_skip}
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_igemm_gpu.py \
  tests/test_ops_gpu.py > "$OUT/tests.log" 2>&1 || exit $?
for v in 1 0 1; do
  RTSEG_SKIP_HANDOFF=$v timeout -k 10 300 python3 -u bench.py --no-infer >> "$OUT/bench_s$v.json" 2>> "$OUT/bench.err" || exit $?
done
RTSEG_PROBE_OPS="$OUT/step_ops.txt" timeout -k 10 300 python3 -u bench.py --no-infer --steps 3 --warmup 2 \
  > "$OUT/probe.json" 2> "$OUT/probe.err"
