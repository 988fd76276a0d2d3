#!/bin/bash
# record the autotune decisions of the BASELINE config 3/4 stand-ins (BiSeNetV2 b16, STDC2 + detail
# head b16) into a copy of the tuning database, then re-run both from that database (warm-up check)
OUT=${1:-gpurun_out/r5_tunedb}
mkdir -p "$OUT"
cp miopen_db/rtseg_conv_decisions.json "$OUT/tune.json"
export RTSEG_TUNE_DB_OUT="$OUT/tune.json"
timeout -k 10 500 python3 -u bench.py --model stdc --arch stdc2 --detail-head --batch 16 --no-infer \
  > "$OUT/stdc2_tune.json" 2> "$OUT/stdc2_tune.err" || exit $?
timeout -k 10 400 python3 -u bench.py --model bisenetv2 --batch 16 --no-infer > "$OUT/bisenetv2_tune.json" \
  2> "$OUT/bisenetv2_tune.err" || exit $?
timeout -k 10 400 python3 -u bench.py --model stdc --arch stdc2 --batch 16 --no-infer > "$OUT/stdc2_aux_tune.json" \
  2> "$OUT/stdc2_aux_tune.err" || exit $?
unset RTSEG_TUNE_DB_OUT
export RTSEG_TUNE_DB="$OUT/tune.json"
timeout -k 10 400 python3 -u bench.py --model stdc --arch stdc2 --detail-head --batch 16 --no-infer \
  > "$OUT/stdc2_db.json" 2> "$OUT/stdc2_db.err" || exit $?
timeout -k 10 400 python3 -u bench.py --model bisenetv2 --batch 16 --no-infer > "$OUT/bisenetv2_db.json" \
  2> "$OUT/bisenetv2_db.err"
