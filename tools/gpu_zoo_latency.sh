#!/bin/bash
# Batch-1 inference latency breakdown of zoo models (the reference README protocol: 1024 x 512,
# tools/test_speed.py), fp32 and bf16: host-timed FPS without the profiler, then a rocprofv3 kernel
# trace analysed by tools/latency_report.py (kernels per forward, kernel time vs replay span vs
# gaps, duration histogram, top kernels).
# usage: tools/gpu_zoo_latency.sh OUT model[,model...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${1:-zoo_latency}; MODELS=${2:-espnet,regseg,fpenet}
mkdir -p $OUT
for m in ${MODELS//,/ }; do
  for p in fp32 bf16; do
    flag=""; [ $p = fp32 ] && flag="--fp32"
    timeout -k 10 180 python3 tools/profile_infer.py --model $m --h 512 --w 1024 --iters 200 $flag > $OUT/${m}_${p}_wall.txt 2>&1 || { tail -5 $OUT/${m}_${p}_wall.txt; exit 1; }
    wall=$(grep -o "[0-9.]* ms/img" $OUT/${m}_${p}_wall.txt | tail -1 | cut -d' ' -f1)
    RAW=/tmp/rtseg_lat_${m}_$p; rm -rf $RAW
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $RAW -o run -- python3 tools/profile_infer.py --model $m --h 512 --w 1024 --iters 200 $flag > $OUT/${m}_${p}_prof.log 2>&1 || { tail -5 $OUT/${m}_${p}_prof.log; exit 1; }
    TRACE=$(find $RAW -name "*kernel_trace.csv" | head -1)
    python3 tools/latency_report.py "$TRACE" --iters 200 --wall-ms "$wall" > $OUT/${m}_${p}.txt || exit 1
    echo "== $m $p: $(tail -1 $OUT/${m}_${p}_wall.txt)"; head -4 $OUT/${m}_${p}.txt
    rm -rf $RAW
  done
done
