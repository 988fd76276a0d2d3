#!/bin/bash
# whalo2 on the headline: bench once re-timing the shapes whose candidate set gained whalo2
# (decisions merged into OUT/tune.json), then the steady number from that database, then the
# A/B with whalo2 off (the in-tree database's round-4 decisions), then a kernel profile.
OUT=${1:-gpurun_out/r5_wh2}
mkdir -p "$OUT"
RTSEG_TUNE_DB_OUT="$OUT/tune.json" timeout -k 10 400 python3 -u bench.py --no-infer > "$OUT/bench_tune.json" 2> "$OUT/tune.err" || exit $?
RTSEG_TUNE_DB="$OUT/tune.json" timeout -k 10 300 python3 -u bench.py --no-infer > "$OUT/bench_on.json" 2> "$OUT/on.err" || exit $?
RTSEG_CONV_WHALO2=0 timeout -k 10 300 python3 -u bench.py --no-infer > "$OUT/bench_off.json" 2> "$OUT/off.err" || exit $?
RTSEG_TUNE_DB="$OUT/tune.json" tools/profile_bench.sh "$OUT/prof" --steps 6 --warmup 3
