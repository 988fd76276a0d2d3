#!/bin/bash
# current-tree training throughput of the other BASELINE configs on one GPU (BiSeNetV2 + aux,
# STDC2 + detail head, batch 16) for the README table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${MODELS_OUT:-models}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --model bisenetv2 --batch 16 --steps 20 --warmup 5 --no-infer \
  > $OUT/bench_bisenetv2_b16.json 2> $OUT/bisenetv2.err || { tail -20 $OUT/bisenetv2.err; exit 1; }
tail -1 $OUT/bench_bisenetv2_b16.json | cut -c1-200
timeout -k 10 300 python -u bench.py --model stdc --arch stdc2 --detail-head --batch 16 --steps 20 --warmup 5 --no-infer \
  > $OUT/bench_stdc2_detail_b16.json 2> $OUT/stdc2.err || { tail -20 $OUT/stdc2.err; exit 1; }
tail -1 $OUT/bench_stdc2_detail_b16.json | cut -c1-200
