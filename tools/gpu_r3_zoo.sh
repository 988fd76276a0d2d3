#!/bin/bash
# Zoo training throughput (tools/zoo_train.py, batch 8 @ 1024x2048) for the models in $ZOO_MODELS,
# with MIOpen's find database and our conv tuning database written under gpurun_out/miopen_db
# (copied back into the tree's miopen_db/ afterwards, so later processes skip the searches).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/miopen_db gpurun_out/r3_zoo
cp -n miopen_db/* gpurun_out/miopen_db/ 2>/dev/null
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/gpurun_out/miopen_db
export RTSEG_TUNE_DB=$GRAFT_REPO_ROOT/gpurun_out/miopen_db/rtseg_conv_decisions.json
export RTSEG_TUNE_DB_OUT=$RTSEG_TUNE_DB
timeout -k 10 ${ZOO_TIMEOUT:-1000} python -u tools/zoo_train.py --batch 8 --steps 5 --warmup 3 --models "$ZOO_MODELS" \
  --out gpurun_out/r3_zoo/zoo_train.jsonl > gpurun_out/r3_zoo/log_${ZOO_TAG:-x}.txt 2>&1
rc=$?
grep "^{" gpurun_out/r3_zoo/log_${ZOO_TAG:-x}.txt | cut -c1-200
exit $rc
