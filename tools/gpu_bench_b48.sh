#!/bin/bash
# the headline bench once more on a fresh box, then batch 48 (per-GPU work x1.5)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/b48
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-infer > $OUT/bench_b32.json 2> $OUT/b32.err || { tail -20 $OUT/b32.err; exit 1; }
tail -1 $OUT/bench_b32.json | cut -c1-250
RTSEG_STACK_DUMP=60 timeout -k 10 400 python -u bench.py --batch 48 --steps 10 --warmup 3 --no-infer \
  > $OUT/bench_b48.json 2> $OUT/b48.err || { grep -v "^  File\|^Thread" $OUT/b48.err | tail -20; exit 1; }
tail -1 $OUT/bench_b48.json | cut -c1-250
