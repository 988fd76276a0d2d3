#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c14
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -v -s --timeout 250 --timeout-method thread -m gpu tests/test_ddp_model_gpu.py "tests/test_routed_conv_gpu.py::test_biased_conv_bias_add_matches_conv2d" > $OUT/tests.log 2>&1
rc=$?; grep -E "passed|failed|Error|vs fp32" $OUT/tests.log | tail -8; if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpu_zoo_sweep.sh B aglnet,lednet,contextnet,fddwnet,dabnet,cfpnet,adscnet adscnet,aglnet,bisenetv1,bisenetv2,canet,cfpnet,cgnet,contextnet,dabnet,ddrnet
