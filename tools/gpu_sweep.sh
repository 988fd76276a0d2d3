#!/bin/bash
# numerics of every tile configuration, then the fwd/dgrad/wgrad config sweep vs MIOpen
mkdir -p gpurun_out
T="timeout -k 10 200 python -u -m pytest tests/test_conv_igemm_gpu.py -x -q --timeout 60 --timeout-method thread"
$T > gpurun_out/t_sweep.log 2>&1 || { tail -30 gpurun_out/t_sweep.log; exit 1; }
for c in 0 1 2 3 4; do RTSEG_IGEMM_CFG=$c $T -k "forward or dgrad" >> gpurun_out/t_sweep.log 2>&1 || { echo "cfg $c failed"; tail -30 gpurun_out/t_sweep.log; exit 1; }; done
for c in 0 1 2 3 4 5; do RTSEG_WGRAD_CFG=$c $T -k "wgrad" >> gpurun_out/t_sweep.log 2>&1 || { echo "wcfg $c failed"; tail -30 gpurun_out/t_sweep.log; exit 1; }; done
grep -E "passed|failed" gpurun_out/t_sweep.log
timeout -k 10 900 python -u tools/bench_conv.py --batch 32 --iters 10 --cfgs 0,1,2,3,4 --wcfgs 0,1,2,3,4,5 > gpurun_out/sweep2.log 2>&1
rc=$?; cat gpurun_out/sweep2.log | grep -v amdgpu.ids
exit $rc
