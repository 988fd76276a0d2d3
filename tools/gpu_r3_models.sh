#!/bin/bash
# BASELINE configs 3/4 on one GPU (BiSeNetV2 + aux, STDC2 + detail head, batch 16): bench +
# rocprofv3 steady-state profile each -> gpurun_out/r3_models/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
# SPECS="tag:losses_per_step:bench args;..." overrides the default pair
IFS=";" read -ra SPECS <<< "${SPECS:-bisenetv2_b16:5:--model bisenetv2 --batch 16;stdc2_detail_b16:1:--model stdc --arch stdc2 --detail-head --batch 16}"
for spec in "${SPECS[@]}"; do
  tag=${spec%%:*}; rest=${spec#*:}; per=${rest%%:*}; args=${rest#*:}
  OUT=gpurun_out/r3_models/$tag
  mkdir -p $OUT
  if [ -z "$NOBENCH" ]; then
    timeout -k 10 300 python -u bench.py $args --steps 20 --warmup 5 --no-infer > $OUT/bench.json 2> $OUT/bench.err \
      || { tail -20 $OUT/bench.err; exit 1; }
    tail -1 $OUT/bench.json | cut -c1-260
  fi
  PROF_SKIP=8 PROF_PER_STEP=$per timeout -k 10 400 bash tools/profile_bench.sh $OUT $args --steps 6 --warmup 5 \
    > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  head -${HEADN:-30} $OUT/steady.txt | cut -c1-170
done
