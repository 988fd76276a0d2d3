#!/bin/bash
# Round 3, call B: fused-optimizer differential tests + zoo gradient-error probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3_b
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fused_optim_gpu.py \
  > gpurun_out/r3_b/fused_optim.log 2>&1
rc=$?
tail -15 gpurun_out/r3_b/fused_optim.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u tools/probe_zoo_gpu_err.py adscnet bisenetv2 dfanet lite_hrnet mininetv2 ppliteseg stdc \
  > gpurun_out/r3_b/zoo_err.log 2>&1
rc=$?
grep -v Warn gpurun_out/r3_b/zoo_err.log | tail -20
exit $rc
