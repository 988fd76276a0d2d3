#!/bin/bash
# Headline bench with the in-tree tuning database vs a fresh per-shape autotune (RTSEG_TUNE_DB=none),
# the fresh decisions written to OUTDIR/tune_fresh.json
OUT=${1:-gpurun_out/r5_retune}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u bench.py --no-infer > "$OUT/bench_db.json" 2> "$OUT/db.err" || exit $?
RTSEG_TUNE_DB=none RTSEG_TUNE_DB_OUT="$OUT/tune_fresh.json" timeout -k 10 400 python3 -u bench.py --no-infer \
  > "$OUT/bench_fresh.json" 2> "$OUT/fresh.err" || exit $?
RTSEG_TUNE_DB="$OUT/tune_fresh.json" timeout -k 10 300 python3 -u bench.py --no-infer > "$OUT/bench_fresh2.json" 2> "$OUT/fresh2.err"
