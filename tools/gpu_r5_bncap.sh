#!/bin/bash
# A/B of the BN streaming-pass grid caps (tools/bench_bn_bw.py), one process per setting.
OUT=${1:-gpurun_out/r5_bncap}
mkdir -p "$OUT"
for c in 1024 2048 4096 16384; do
  RTSEG_BN_APPLY_CAP=$c timeout -k 10 120 python3 -u tools/bench_bn_bw.py --reps 10 > "$OUT/apply_cap$c.txt" 2>&1 || exit $?
done
for c in 512 2048 4096; do
  RTSEG_BN_REDUCE_CAP=$c timeout -k 10 120 python3 -u tools/bench_bn_bw.py --reps 10 > "$OUT/reduce_cap$c.txt" 2>&1 || exit $?
done
