#!/bin/bash
# BN pass traversal order vs the Infinity Cache (RTSEG_BN_L3ORDER, csrc/kernels/bn_act.hip):
# BN numerics under the non-default orders, then the headline bench per order.
# usage: tools/gpu_r5_l3order.sh OUTDIR [tuning-db]
OUT=${1:-gpurun_out/r5_l3}
[ -n "$2" ] && export RTSEG_TUNE_DB="$2"
mkdir -p "$OUT"
for o in 5 10; do
  RTSEG_BN_L3ORDER=$o timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_bn_gpu.py > "$OUT/test_bn_$o.log" 2>&1 || exit $?
done
for o in 0 1 9 6 14 0; do
  RTSEG_BN_L3ORDER=$o timeout -k 10 300 python3 -u bench.py --no-infer >> "$OUT/bench_$o.json" 2>> "$OUT/bench_$o.err" || exit $?
done
