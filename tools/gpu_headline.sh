#!/bin/bash
# headline run: bench on a fresh tuning DB (written for commit), a second process on it,
# the steady-state profile, one batch-48 run (the round-2 "hang", now bounded autotune)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${HEADLINE_OUT:-headline}
mkdir -p $OUT
RTSEG_TUNE_DB=none RTSEG_TUNE_DB_OUT=$OUT/rtseg_conv_decisions.json RTSEG_DECISIONS_OUT=$OUT/decisions.txt \
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-1300
RTSEG_TUNE_DB=$OUT/rtseg_conv_decisions.json timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-infer \
  > $OUT/bench_db.json 2> $OUT/bench_db.err || { tail -20 $OUT/bench_db.err; exit 1; }
tail -1 $OUT/bench_db.json | cut -c1-300
RTSEG_TUNE_DB=$OUT/rtseg_conv_decisions.json PROF_SKIP=8 PROF_PER_STEP=2 timeout -k 10 500 bash tools/profile_bench.sh $OUT --steps 6 --warmup 5 \
  > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
rm -f $OUT/trace.csv.gz
head -40 $OUT/steady.txt | cut -c1-170
RTSEG_TUNE_DB=$OUT/rtseg_conv_decisions.json RTSEG_STACK_DUMP=60 timeout -k 10 400 python -u bench.py --batch 48 --steps 5 --warmup 3 --no-infer \
  > $OUT/bench_b48.json 2> $OUT/bench_b48.err || { grep -v "^  File\|^Thread" $OUT/bench_b48.err | tail -20; exit 1; }
tail -1 $OUT/bench_b48.json | cut -c1-400
