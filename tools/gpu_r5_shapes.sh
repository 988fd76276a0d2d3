#!/bin/bash
# Round 5: first-step cost at new shapes and the KD config (BASELINE config 5).
# usage (GPU box): bash tools/gpu_r5_shapes.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5_shapes}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u bench.py --batch 48 --steps 5 --warmup 2 --no-infer > "$OUT/b48.json" 2> "$OUT/b48.err" || exit $?
timeout -k 10 300 python3 -u bench.py --height 512 --width 1024 --steps 5 --warmup 2 --no-infer > "$OUT/h512.json" 2> "$OUT/h512.err" || exit $?
timeout -k 10 300 python3 -u bench.py --kd --batch 16 --steps 10 --warmup 3 --no-infer > "$OUT/kd_b16.json" 2> "$OUT/kd_b16.err" || exit $?
PROF_SKIP=4 bash tools/profile_bench.sh "$OUT/kd_prof" --kd --batch 16 --steps 6 --warmup 3
