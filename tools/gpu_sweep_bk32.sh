#!/bin/bash
# numerics of the BK=32 deep-ring tile configs (5, 6, 7), then fwd/dgrad timing vs the BK=64 ones
mkdir -p gpurun_out
T="timeout -k 10 200 python -u -m pytest tests/test_conv_igemm_gpu.py -x -q --timeout 60 --timeout-method thread"
for c in 5 6 7; do RTSEG_IGEMM_CFG=$c $T -k "forward or dgrad" >> gpurun_out/t_bk32.log 2>&1 || { echo "cfg $c failed"; tail -30 gpurun_out/t_bk32.log; exit 1; }; done
grep -E "passed|failed" gpurun_out/t_bk32.log
timeout -k 10 600 python -u tools/bench_conv.py --batch 32 --iters 10 --only fwd,dgrad --cfgs 2,3,4,5,6,7 > gpurun_out/sweep_bk32.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/sweep_bk32.log
exit $rc
