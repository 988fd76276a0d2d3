#!/bin/bash
# round 4: DDP rehearsal (first-update comparison), PSP-model numerics, zoo sweep chunk A
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c11
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_ddp_model_gpu.py > $OUT/ddp.log 2>&1
rc=$?; grep -E "amp=|passed|failed" $OUT/ddp.log | cut -c1-300; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_zoo.py -k "fastscnn or icnet or espnetv2 or swiftnet" > $OUT/ppm.log 2>&1
rc=$?; tail -2 $OUT/ppm.log; if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpu_zoo_sweep.sh A adscnet,aglnet,bisenetv1,bisenetv2,canet,cfpnet,cgnet,contextnet,dabnet
