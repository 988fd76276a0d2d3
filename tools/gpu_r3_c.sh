#!/bin/bash
# Round 3, call C: new zoo numerics checks (frozen-BN + train-BN vs fp64) in a plain process.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3_c
export PYTHONUNBUFFERED=1
export ZOO_ONLY=${ZOO_ONLY:-lednet,regseg,liteseg,bisenetv2,stdc,ddrnet,enet,cgnet}
timeout -k 10 500 python -u tests/isolated/zoo_gpu_check.py > gpurun_out/r3_c/zoo.log 2>&1
rc=$?
grep -E "FAILED|ok$|skipped|done|Error" gpurun_out/r3_c/zoo.log | head -40
grep -E "AssertionError" gpurun_out/r3_c/zoo.log | head -20
exit $rc
