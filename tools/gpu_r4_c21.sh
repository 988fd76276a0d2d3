#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c21
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_routed_conv_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
bash tools/gpu_zoo_sweep.sh G regseg,bisenetv1,bisenetv2,canet,cgnet,farseenet,fastscnn,espnetv2 - || exit 1
TRAIN_TIMEOUT=330 bash tools/gpu_zoo_sweep.sh H segnet -
