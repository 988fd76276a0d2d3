#!/bin/bash
# BN-backward reduction in the dgrad epilogue: kernel + model tests, numerics, bench/profile
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_train_numerics_gpu.py tests/test_deconv_unpool_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_c15.log 2>&1
rc=$?; grep -E "FAIL|Error|rror:|passed|failed" gpurun_out/t_c15.log | cut -c1-200 | tail -30
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench.sh b32
