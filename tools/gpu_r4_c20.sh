#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c20
mkdir -p $OUT
timeout -k 10 300 python -u tools/probe_grouped_conv.py > $OUT/grouped.txt 2>&1 || { tail -20 $OUT/grouped.txt; exit 1; }
cat $OUT/grouped.txt
bash tools/gpu_zoo_sweep.sh F fpenet,segnet,bisenetv1,bisenetv2,canet,cgnet,farseenet,fastscnn,espnetv2 -
