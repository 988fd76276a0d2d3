#!/bin/bash
# one GPU call: the whole one-process GPU suite (as the driver runs it), smoke(), then the
# steady-state rocprofv3 profile of the headline step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${SUITE_OUT:-suite}
mkdir -p $OUT
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -4 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -12; exit $rc; }
PROF_OUT=${SUITE_OUT:-suite}/prof bash tools/gpu_prof.sh
