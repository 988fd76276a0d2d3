#!/bin/bash
# full GPU test suite, then bf16 vs fp32 inference kernels of the models whose bf16 FPS trails fp32
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/r4_c25
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|error" $OUT/pytest_gpu.log | tail -20; exit $rc; }
for m in espnetv2 dfanet fastscnn; do
  for p in bf16 fp32; do
    flag=""; [ $p = fp32 ] && flag="--fp32"
    RAW=/tmp/rtseg_inf_${m}_$p
    rm -rf $RAW
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $RAW -o run -- \
      python3 tools/profile_infer.py --model $m --h 512 --w 1024 --iters 100 $flag > $OUT/${m}_$p.log 2>&1 || { tail -20 $OUT/${m}_$p.log; exit 1; }
    STATS=$(find $RAW -name "*kernel_stats.csv" | head -1)
    python3 tools/summarize_kernel_stats.py $STATS > $OUT/${m}_$p.txt
    grep FPS $OUT/${m}_$p.log
  done
done
