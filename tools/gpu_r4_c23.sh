#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r4_c23
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_routed_conv_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
TRAIN_TIMEOUT=600 bash tools/gpu_zoo_sweep.sh I espnetv2,regseg,segnet - || exit 1
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
