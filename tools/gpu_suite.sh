#!/bin/bash
# One GPU call in the driver's form: smoke(), then the one-process GPU suite (all of tests/ -m gpu,
# or the pytest arguments given), then optionally (PROF=1) the steady-state profile of the
# headline step.  A crash, abort or time limit ends the call there.
# usage: tools/gpu_suite.sh OUT [pytest args...]      (OUT under gpurun_out/)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${1:-suite}; shift || true
mkdir -p $OUT
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
ARGS=("$@"); [ ${#ARGS[@]} -eq 0 ] && ARGS=(tests -m gpu)
timeout -k 10 ${SUITE_TIMEOUT:-900} python -u -m pytest "${ARGS[@]}" -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -4 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -12; exit $rc; }
[ -n "$PROF" ] && PROF_OUT=${OUT#gpurun_out/}/prof bash tools/gpu_prof.sh
exit 0
