#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c19
mkdir -p $OUT
PROF_SKIP=3 PROF_PER_STEP=1 timeout -k 10 300 bash tools/profile_bench.sh $OUT/fpenet --model fpenet --batch 8 --steps 2 --warmup 3 \
  > $OUT/fpenet.log 2>&1 || { tail -20 $OUT/fpenet.log; exit 1; }
rm -f $OUT/fpenet/trace.csv.gz $OUT/fpenet/kernel_stats.csv
head -30 $OUT/fpenet/steady.txt | cut -c1-190
bash tools/gpu_zoo_sweep.sh E mininet,mininetv2,ppliteseg,regseg,segnet,shelfnet,sqnet,stdc,swiftnet -
