#!/bin/bash
# End-of-round verification on one MI355X: the whole GPU suite in ONE pytest process, smoke(), the
# headline bench and a rocprofv3 steady-state profile of it -> gpurun_out/r3_final/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r3_final
mkdir -p $OUT
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 780 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; grep -E "^FAILED|^ERROR" $OUT/pytest_gpu.log | head; [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -10 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-400
PROF_SKIP=8 PROF_PER_STEP=2 timeout -k 10 300 bash tools/profile_bench.sh $OUT --steps 6 --warmup 5 > $OUT/prof.log 2>&1 \
  || { tail -10 $OUT/prof.log; exit 1; }
head -40 $OUT/steady.txt | cut -c1-170
