#!/bin/bash
# staggered DMA issue (RTSEG_IGEMM_STAGGER=1): numerics, then fwd/dgrad timing with and without
mkdir -p gpurun_out
RTSEG_IGEMM_STAGGER=1 timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py -x -q --timeout 60 --timeout-method thread > gpurun_out/st_test.log 2>&1 || { tail -30 gpurun_out/st_test.log; exit 1; }
tail -1 gpurun_out/st_test.log
timeout -k 10 300 python -u tools/bench_conv.py --batch 32 --iters 10 --only fwd,dgrad --shapes 0,1,2,3,4,5,6 > gpurun_out/st_off.log 2>&1 || { tail -20 gpurun_out/st_off.log; exit 1; }
RTSEG_IGEMM_STAGGER=1 timeout -k 10 300 python -u tools/bench_conv.py --batch 32 --iters 10 --only fwd,dgrad --shapes 0,1,2,3,4,5,6 > gpurun_out/st_on.log 2>&1 || { tail -20 gpurun_out/st_on.log; exit 1; }
paste <(grep -E "fwd |dgrad " gpurun_out/st_off.log | awk '{print $1, $2, $5}') <(grep -E "fwd |dgrad " gpurun_out/st_on.log | awk '{print $5}')
