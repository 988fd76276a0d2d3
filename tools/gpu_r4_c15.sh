#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c15
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v -s --timeout 250 --timeout-method thread -m gpu "tests/test_ddp_model_gpu.py::test_ddp_two_ranks_match_one_process[ddrnet23slim_aux]" tests/test_ops_gpu.py -k "ddrnet or ohem or ce_loss or loss" > $OUT/tests.log 2>&1
rc=$?; grep -E "passed|failed|vs fp32" $OUT/tests.log | tail -5; if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpu_zoo_sweep.sh C ddrnet,dfanet,edanet,enet,erfnet,esnet,espnet bisenetv1,dfanet,edanet,enet,erfnet,esnet,espnet,espnetv2,farseenet,fastscnn,fddwnet,fpenet,fssnet,icnet
