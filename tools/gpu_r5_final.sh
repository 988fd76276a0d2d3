#!/bin/bash
# round-5 closing numbers: the driver's default bench (training + inference), BASELINE configs 3/4
# single-GPU stand-ins (BiSeNetV2 + aux, STDC2 + detail head, batch 16), KD (config 5), and a
# steady-state profile of the headline step
OUT=${1:-gpurun_out/r5_final}
mkdir -p "$OUT"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
timeout -k 10 400 python3 -u bench.py --model bisenetv2 --batch 16 --no-infer > "$OUT/bench_bisenetv2_b16.json" \
  2> "$OUT/bench_bisenetv2.err" || exit $?
timeout -k 10 400 python3 -u bench.py --model stdc --arch stdc2 --detail-head --batch 16 --no-infer \
  > "$OUT/bench_stdc2_detail_b16.json" 2> "$OUT/bench_stdc2.err" || exit $?
timeout -k 10 400 python3 -u bench.py --kd --batch 16 --no-infer > "$OUT/bench_kd_b16.json" 2> "$OUT/bench_kd.err" || exit $?
tools/profile_bench.sh "$OUT/prof" --steps 6 --warmup 3
