#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (run on the GPU box).
# usage: tools/profile_bench.sh OUTDIR [bench args...]
set -e
OUT=${1:-gpurun_out/prof}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 bench.py --no-infer "$@" > "$OUT/bench.log" 2>&1
find "$OUT" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$OUT/kernel_stats.csv"
python3 tools/summarize_kernel_stats.py "$OUT/kernel_stats.csv" > "$OUT/summary.txt"
