#!/bin/bash
# addend-aware dgrad keys: re-record the tuning database for the headline and the config 3/4 stand-ins,
# then the headline from that database
OUT=${1:-gpurun_out/r5_addkey}
mkdir -p "$OUT"
cp miopen_db/rtseg_conv_decisions.json "$OUT/tune.json"
export RTSEG_TUNE_DB_OUT="$OUT/tune.json" RTSEG_DECISIONS_OUT="$OUT/decisions_ddrnet.tsv"
timeout -k 10 400 python3 -u bench.py --no-infer > "$OUT/ddrnet_tune.json" 2> "$OUT/ddrnet_tune.err" || exit $?
unset RTSEG_DECISIONS_OUT
timeout -k 10 400 python3 -u bench.py --model bisenetv2 --batch 16 --no-infer > "$OUT/bisenetv2_tune.json" 2> "$OUT/b.err" || exit $?
timeout -k 10 400 python3 -u bench.py --model stdc --arch stdc2 --detail-head --batch 16 --no-infer \
  > "$OUT/stdc2_tune.json" 2> "$OUT/s.err" || exit $?
timeout -k 10 400 python3 -u bench.py --model stdc --arch stdc2 --batch 16 --no-infer > "$OUT/stdc2aux_tune.json" \
  2> "$OUT/s2.err" || exit $?
unset RTSEG_TUNE_DB_OUT
export RTSEG_TUNE_DB="$OUT/tune.json"
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-infer >> "$OUT/ddrnet_db.json" 2>> "$OUT/ddrnet_db.err" || exit $?
done
