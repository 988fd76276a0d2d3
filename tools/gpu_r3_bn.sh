#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3_bn
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_syncbn_gpu.py \
  "tests/test_bn_gpu.py::test_fused_batchnorm_module_matches_torch" tests/test_dwconv_gpu.py > gpurun_out/r3_bn/log.txt 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|Mismatch|Greatest" gpurun_out/r3_bn/log.txt | grep -v "test_dwconv_fwd_bwd" | head -40
exit $rc
