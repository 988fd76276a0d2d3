#!/bin/bash
# rocprofv3 kernel trace of the bench step (b32) -> gpurun_out/r3_prof, plus the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r3_prof
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-700
PROF_SKIP=8 PROF_PER_STEP=2 timeout -k 10 600 bash tools/profile_bench.sh $OUT --steps 6 --warmup 5 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
head -60 $OUT/steady.txt | cut -c1-180
