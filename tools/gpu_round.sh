#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_detail_loss_gpu.py tests/test_conv_gpu.py > gpurun_out/t_detail.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_detail.log; exit 1; }
tail -2 gpurun_out/t_detail.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 5 --batch 16 --model stdc --arch stdc2 --detail-head --no-infer > gpurun_out/b_stdc.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/b_stdc.log; exit 1; }
tail -1 gpurun_out/b_stdc.log
