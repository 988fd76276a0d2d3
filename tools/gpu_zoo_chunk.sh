#!/bin/bash
# One chunk of the zoo training-throughput sweep (tools/zoo_train.py), conv decisions merged into
# gpurun_out/zoo_db.json (copy it into miopen_db/rtseg_conv_decisions.json afterwards).
# usage: tools/gpu_zoo_chunk.sh TAG model,model,...   (PRE="cmd" runs a short step first)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
TAG=$1; MODELS=$2
mkdir -p gpurun_out/zoo
if [ -n "$PRE" ]; then bash -c "$PRE" || exit 1; fi
RTSEG_TUNE_DB_OUT=gpurun_out/zoo_db.json timeout -k 10 ${ZOO_T:-1000} python -u tools/zoo_train.py --batch 8 --steps 5 --warmup 3 \
  --models "$MODELS" --out gpurun_out/zoo/train_$TAG.jsonl > gpurun_out/zoo/train_$TAG.log 2>&1
rc=$?
cut -c1-200 gpurun_out/zoo/train_$TAG.jsonl
exit $rc
