#!/bin/bash
# rocprofv3 steady-state profile of the headline step (extra env passed through: e.g. the A/B
# switches), written to gpurun_out/$PROF_OUT
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${PROF_OUT:-prof}
mkdir -p $OUT
PROF_SKIP=8 PROF_PER_STEP=2 timeout -k 10 500 bash tools/profile_bench.sh $OUT --steps 6 --warmup 5 \
  > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
rm -f $OUT/trace.csv.gz
head -45 $OUT/steady.txt | cut -c1-160
