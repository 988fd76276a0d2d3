#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c18
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_fused_optim_gpu.py tests/test_routed_conv_gpu.py tests/test_concat_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; grep -E "^E " $OUT/tests.log | head -10
timeout -k 10 200 python -u tools/probe_ema_determinism.py > $OUT/ema_probe.log 2>&1; grep -E "mismatched|Error" $OUT/ema_probe.log
RTSEG_CONCAT_SINK=0 timeout -k 10 200 python -u tools/probe_ema_determinism.py > $OUT/ema_probe_nosink.log 2>&1; grep -E "mismatched|Error" $OUT/ema_probe_nosink.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_zoo_sweep.sh D2 esnet,fpenet,fssnet,icnet,linknet,lite_hrnet,liteseg -
