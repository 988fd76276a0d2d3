#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_syncbn_gpu.py tests/test_train_numerics_gpu.py tests/test_deconv_unpool_gpu.py tests/test_conv_igemm_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/t_new.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|rror:" gpurun_out/t_new.log | cut -c1-200 | tail -60
exit $rc
