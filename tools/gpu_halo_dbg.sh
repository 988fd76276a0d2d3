#!/bin/bash
# halo conv: numerics + timing sweeps over the tile configs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/halo_pytest.log 2>&1 || { echo TFAIL; tail -40 gpurun_out/halo_pytest.log; exit 1; }
tail -2 gpurun_out/halo_pytest.log
timeout -k 10 300 python -u tools/bench_conv.py --only fwd,dgrad --shapes 0,2,4,6 --iters 30 > gpurun_out/hdbg0.txt 2>&1 || { tail -20 gpurun_out/hdbg0.txt; exit 1; }
RTSEG_HALO_CFG=1 timeout -k 10 200 python -u tools/bench_conv.py --only fwd --shapes 2,4 --iters 30 > gpurun_out/hdbg1.txt 2>&1 || { tail -20 gpurun_out/hdbg1.txt; exit 1; }
cat gpurun_out/hdbg0.txt; grep halo gpurun_out/hdbg1.txt
