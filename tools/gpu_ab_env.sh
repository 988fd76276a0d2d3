#!/bin/bash
# Same-box A/B of one bench configuration under two environment settings (alternating A B A B).
# usage: tools/gpu_ab_env.sh TAG "ENV_A" "ENV_B" [bench args...]   e.g. "RTSEG_CONCAT_SINK=0" ""
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1; A=$2; B=$3; shift 3
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for r in 1 2; do
  for side in A B; do
    [ $side = A ] && E=$A || E=$B
    env $E timeout -k 10 300 python -u bench.py "$@" > $OUT/${side}$r.json 2> $OUT/${side}$r.err \
      || { tail -20 $OUT/${side}$r.err; exit 1; }
    echo "$side$r [$E] $(tail -1 $OUT/${side}$r.json | cut -c1-120)"
  done
done
