#!/bin/bash
# gate kernels + zoo models using them, then BiSeNetV2 b16 bench/profile
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gate_gpu.py tests/test_zoo.py -x -q --timeout 300 --timeout-method thread -k "gate or bisenet or regseg or cgnet or canet or pp_lite or aglnet or lite_hrnet" > gpurun_out/t_c19.log 2>&1
rc=$?; grep -E "FAIL|Error|rror:|passed|failed" gpurun_out/t_c19.log | cut -c1-200 | tail -20
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench.sh bisev2_b16 --model bisenetv2 --batch 16 --no-infer
