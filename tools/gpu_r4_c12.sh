#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
bash tools/gpu_zoo_sweep.sh B contextnet,dabnet,ddrnet,dfanet,edanet,enet adscnet,aglnet,bisenetv1,bisenetv2,canet,cfpnet,cgnet,contextnet,dabnet
