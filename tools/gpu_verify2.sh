#!/bin/bash
# New kernel tests first, then the round-end style verification (GPU suite, smoke, bench).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_act_gpu.py tests/test_shuffle_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/v2_new.log 2>&1 || { echo NFAIL; tail -30 gpurun_out/v2_new.log; exit 1; }
tail -2 gpurun_out/v2_new.log
bash tools/gpu_verify.sh
