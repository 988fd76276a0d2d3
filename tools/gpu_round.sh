#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW=0
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_bn_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t1.log; exit 1; }
tail -1 gpurun_out/t1.log
rm -rf /tmp/rtseg_infer_raw
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rtseg_infer_raw -o run -- python3 tools/profile_infer.py > gpurun_out/infer_prof.log 2>&1 || { echo INFERFAIL; tail -30 gpurun_out/infer_prof.log; exit 1; }
grep FPS gpurun_out/infer_prof.log
STATS=$(find /tmp/rtseg_infer_raw -name "*kernel_stats.csv" | head -1)
mkdir -p gpurun_out/prof_infer && cp "$STATS" gpurun_out/prof_infer/kernel_stats.csv
python3 tools/summarize_kernel_stats.py gpurun_out/prof_infer/kernel_stats.csv > gpurun_out/prof_infer/summary.txt
head -30 gpurun_out/prof_infer/summary.txt
timeout -k 10 300 python3 tools/profile_infer.py > gpurun_out/infer.log 2>&1 && grep FPS gpurun_out/infer.log
