#!/bin/bash
# Round-end style verification on one MI355X: GPU tests, smoke(), default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 780 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v_pytest.log 2>&1 || { echo TFAIL; tail -40 gpurun_out/v_pytest.log; exit 1; }
tail -3 gpurun_out/v_pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v_smoke.log 2>&1 || { echo SFAIL; tail -20 gpurun_out/v_smoke.log; exit 1; }
tail -1 gpurun_out/v_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/v_bench.log 2>&1 || { echo BFAIL; tail -20 gpurun_out/v_bench.log; exit 1; }
tail -1 gpurun_out/v_bench.log
