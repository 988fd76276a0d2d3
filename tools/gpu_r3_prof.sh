#!/bin/bash
# Bench step (b32) with the per-shape conv decisions written to a tuning DB, rocprofv3 kernel
# trace of the bench step -> gpurun_out/r3_prof, then the model-level numerics tests.
# B48=1: also one batch-48 bench with Python stack dumps every 60 s (diagnose a slow first step).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r3_prof
mkdir -p $OUT
RTSEG_TUNE_DB=none RTSEG_TUNE_DB_OUT=$OUT/rtseg_conv_decisions.json RTSEG_DECISIONS_OUT=$OUT/decisions.txt \
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-700
RTSEG_TUNE_DB=$OUT/rtseg_conv_decisions.json timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-infer \
  > $OUT/bench_db.json 2> $OUT/bench_db.err || { tail -20 $OUT/bench_db.err; exit 1; }
tail -1 $OUT/bench_db.json | cut -c1-300
RTSEG_TUNE_DB=$OUT/rtseg_conv_decisions.json PROF_SKIP=8 PROF_PER_STEP=2 timeout -k 10 600 bash tools/profile_bench.sh $OUT --steps 6 --warmup 5 \
  > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
head -60 $OUT/steady.txt | cut -c1-180
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1 \
    || { tail -30 $OUT/tests.log; exit 1; }
  grep -E "cos median|passed|failed" $OUT/tests.log
fi
if [ -n "$B48" ]; then
  RTSEG_TUNE_DB=$OUT/rtseg_conv_decisions.json RTSEG_STACK_DUMP=60 timeout -k 10 420 python -u bench.py --batch 48 --steps 10 --warmup 3 --no-infer \
    > $OUT/bench_b48.json 2> $OUT/bench_b48.err || { tail -40 $OUT/bench_b48.err; exit 1; }
  tail -1 $OUT/bench_b48.json | cut -c1-300
fi
