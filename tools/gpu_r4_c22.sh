#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r4_c22
mkdir -p $OUT
PROF_SKIP=2 PROF_PER_STEP=1 timeout -k 10 420 bash tools/profile_bench.sh $OUT/espnetv2 --model espnetv2 --batch 8 --steps 2 --warmup 2 \
  > $OUT/espnetv2.log 2>&1 || { tail -20 $OUT/espnetv2.log; exit 1; }
rm -f $OUT/espnetv2/trace.csv.gz $OUT/espnetv2/kernel_stats.csv
head -40 $OUT/espnetv2/steady.txt | cut -c1-200
timeout -k 10 300 python -u tools/probe_conv_shapes.py --model segnet > $OUT/segnet_shapes.txt 2>&1; rc=$?
cat $OUT/segnet_shapes.txt; [ $rc -ne 0 ] && exit $rc
# bf16 vs fp32 inference kernels of the zoo models whose bf16 FPS trails fp32 (batch 1, 1024x512)
for m in espnetv2 dfanet fastscnn; do
  for p in bf16 fp32; do
    flag=""; [ $p = fp32 ] && flag="--fp32"
    RAW=/tmp/rtseg_inf_${m}_$p
    rm -rf $RAW
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $RAW -o run -- \
      python3 tools/profile_infer.py --model $m --h 512 --w 1024 --iters 100 $flag > $OUT/${m}_$p.log 2>&1 || { tail -20 $OUT/${m}_$p.log; exit 1; }
    STATS=$(find $RAW -name "*kernel_stats.csv" | head -1)
    python3 tools/summarize_kernel_stats.py $STATS > $OUT/${m}_$p.txt
    grep FPS $OUT/${m}_$p.log
  done
done
