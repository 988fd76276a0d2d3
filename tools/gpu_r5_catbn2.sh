#!/bin/bash
# CGNet / EDANet training A/B of ops.cat_bn_act, alternating order after a tuning run
OUT=${1:-gpurun_out/r5_catbn2}
mkdir -p "$OUT"
for v in 1 1 0 1 0; do
  RTSEG_CONCAT_SINK=$v timeout -k 10 400 python3 -u tools/zoo_train.py --models cgnet,edanet --batch 8 --steps 20 \
    --warmup 5 --out "$OUT/zoo_train.jsonl" >> "$OUT/zoo_train.log" 2>&1 || exit $?
  echo "sink=$v" >> "$OUT/zoo_train.jsonl"
done
