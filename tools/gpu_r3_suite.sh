#!/bin/bash
# Whole GPU suite in ONE pytest process (the round-2 fault appeared only there).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3_suite
export PYTHONUNBUFFERED=1
timeout -k 10 1120 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
  > gpurun_out/r3_suite/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/r3_suite/pytest_gpu.log | tail -3
grep -E "FAILED|Error" gpurun_out/r3_suite/pytest_gpu.log | head -10
exit $rc
