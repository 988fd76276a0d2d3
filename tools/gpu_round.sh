#!/bin/bash
# new GPU tests (SyncBN over 2 ranks, model-level numerics) + headline bench + steady profile
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_syncbn_gpu.py tests/test_train_numerics_gpu.py tests/test_conv_igemm_gpu.py tests/test_deconv_unpool_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_new.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/t_new.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_bench.sh b32
