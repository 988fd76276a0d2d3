#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c17
mkdir -p $OUT
timeout -k 10 200 python -u tools/probe_ema_determinism.py > $OUT/ema_probe.log 2>&1; grep -E "mismatched|Error" $OUT/ema_probe.log
RTSEG_CONCAT_SINK=0 timeout -k 10 200 python -u tools/probe_ema_determinism.py > $OUT/ema_probe_nosink.log 2>&1; grep -E "mismatched|Error" $OUT/ema_probe_nosink.log
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_fused_optim_gpu.py tests/test_routed_conv_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; grep -E "^E " $OUT/tests.log | head -10
bash tools/gpu_zoo_sweep.sh D esnet,fpenet,fssnet,icnet,linknet,lite_hrnet,liteseg lednet,linknet,lite_hrnet,liteseg,mininet,mininetv2,ppliteseg,regseg,segnet,shelfnet,sqnet,stdc,swiftnet,espnetv2,fastscnn,dfanet
