#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_train_numerics_gpu.py tests/test_syncbn_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_c14.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|rror:" gpurun_out/t_c14.log | cut -c1-200 | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/probe_train_numerics.py > gpurun_out/probe_num2.log 2>&1 || exit $?
grep -E "losses|min" gpurun_out/probe_num2.log
bash tools/gpu_bench.sh b32
