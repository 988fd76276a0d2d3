#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pool_gpu.py tests/test_ops_gpu.py -k "pool or interp" > gpurun_out/t_ip.log 2>&1 || { echo TFAIL; tail -40 gpurun_out/t_ip.log; exit 1; }
tail -3 gpurun_out/t_ip.log
rm -rf gpurun_out/prof_infer3 /tmp/rtseg_pi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rtseg_pi -o run -- python3 $GRAFT_REPO_ROOT/tools/profile_infer.py --iters 50 > $GRAFT_REPO_ROOT/gpurun_out/pi.log 2>&1 || { echo PFAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pi.log; exit 1; }
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_infer3
cp $(find /tmp/rtseg_pi -name "*kernel_stats.csv" | head -1) gpurun_out/prof_infer3/kernel_stats.csv
python3 tools/summarize_kernel_stats.py gpurun_out/prof_infer3/kernel_stats.csv > gpurun_out/prof_infer3/summary.txt
grep -v amdgpu gpurun_out/pi.log | tail -3
head -30 gpurun_out/prof_infer3/summary.txt | cut -c1-160
timeout -k 10 300 python tools/test_speed.py --model ddrnet --arch_type DDRNet-23 --ratio 1.0 > gpurun_out/ts.log 2>&1 || { echo SFAIL; tail -20 gpurun_out/ts.log; exit 1; }
tail -4 gpurun_out/ts.log
