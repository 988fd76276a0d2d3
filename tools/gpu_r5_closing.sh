#!/bin/bash
# closing evidence: the driver's one-process GPU suite, the default bench (training + inference), a profile
OUT=${1:-gpurun_out/r5_closing}
mkdir -p "$OUT"
timeout -k 10 1000 python3 -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
tools/profile_bench.sh "$OUT/prof" --steps 6 --warmup 3
