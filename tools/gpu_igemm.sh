#!/bin/bash
# conv_igemm numerics + fwd/dgrad/wgrad benchmark vs MIOpen (one GPU call)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_igemm.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/t_igemm.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u tools/bench_conv.py --batch 32 --iters 10 > gpurun_out/bench_conv.log 2>&1
rc=$?
cat gpurun_out/bench_conv.log | tail -40
exit $rc
