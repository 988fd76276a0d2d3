#!/bin/bash
# inference kernels of the zoo models whose bf16 FPS trails fp32 (README zoo table): rocprofv3
# kernel stats at batch 1, 1024x512 (the reference README protocol), bf16 and fp32
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/infer
mkdir -p $OUT
for m in espnetv2 dfanet fastscnn; do
  for p in bf16 fp32; do
    flag=""; [ $p = fp32 ] && flag="--fp32"
    RAW=/tmp/rtseg_inf_${m}_$p
    rm -rf $RAW
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $RAW -o run -- \
      python3 tools/profile_infer.py --model $m --h 512 --w 1024 --iters 100 $flag > $OUT/${m}_$p.log 2>&1 || { tail -20 $OUT/${m}_$p.log; exit 1; }
    STATS=$(find $RAW -name "*kernel_stats.csv" | head -1)
    python3 tools/summarize_kernel_stats.py $STATS > $OUT/${m}_$p.txt
    echo "$m $p: $(grep -i fps $OUT/${m}_$p.log | tail -1)"
  done
done
