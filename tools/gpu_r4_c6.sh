#!/bin/bash
# round 4: new halo conv kernels (tests + A/B bench), then the DDP / convergence tests
mkdir -p gpurun_out/r4_c6
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_wres_gpu.py > gpurun_out/r4_c6/wres_tests.log 2>&1 || exit $?
for c in 0 1 2 3; do
  RTSEG_WRES_CFG=$c timeout -k 10 200 python -u tools/bench_conv.py --shapes 0 --only fwd,dgrad > gpurun_out/r4_c6/bench_wres_cfg$c.txt 2>&1 || exit $?
done
timeout -k 10 300 python -u tools/bench_conv.py --shapes 0,2,4,6 --only wgrad > gpurun_out/r4_c6/bench_wgrad.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v -s --durations=0 --timeout 400 --timeout-method thread -m gpu tests/test_ddp_model_gpu.py tests/test_convergence.py -k "converges or ddp" > gpurun_out/r4_c6/pytest.log 2>&1
