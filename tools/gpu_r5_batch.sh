#!/bin/bash
# Headline-config throughput vs per-GPU batch (288 GB HBM: batch 32 uses 26 GB), recording the
# autotune decisions of each new batch into OUTDIR/tune_bNN.json (RTSEG_TUNE_DB_OUT).
OUT=${1:-gpurun_out/r5_batch}
mkdir -p "$OUT"
for b in 48 64; do
  RTSEG_TUNE_DB_OUT="$OUT/tune_b$b.json" timeout -k 10 400 python3 -u bench.py --batch $b --steps 10 --warmup 3 --no-infer \
    > "$OUT/b$b.json" 2> "$OUT/b$b.err" || exit $?
done
