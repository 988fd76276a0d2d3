#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (run on the GPU box).
# usage: tools/profile_bench.sh OUTDIR [bench args...]
# Leaves OUTDIR/{bench.log,kernel_stats.csv,summary.txt,steady.txt,trace.csv.gz}
set -e
OUT=${1:-gpurun_out/prof}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
RAW=/tmp/rtseg_prof_raw
rm -rf "$RAW"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$RAW" -o run -- \
  python3 bench.py --no-infer "$@" > "$OUT/bench.log" 2>&1
STATS=$(find "$RAW" -name "*kernel_stats.csv" | head -1)
TRACE=$(find "$RAW" -name "*kernel_trace.csv" | head -1)
cp "$STATS" "$OUT/kernel_stats.csv"
python3 tools/summarize_kernel_stats.py "$OUT/kernel_stats.csv" > "$OUT/summary.txt"
python3 tools/summarize_trace.py "$TRACE" --skip "${PROF_SKIP:-3}" --per-step "${PROF_PER_STEP:-2}" --top 60 > "$OUT/steady.txt"
gzip -c "$TRACE" > "$OUT/trace.csv.gz"
ls -la "$OUT"
