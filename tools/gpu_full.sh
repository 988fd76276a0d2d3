#!/bin/bash
# Round-end rehearsal on one MI355X: every GPU test, smoke(), default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tgpu_full.log 2>&1 || { echo TFAIL; tail -40 gpurun_out/tgpu_full.log; exit 1; }
tail -2 gpurun_out/tgpu_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo BFAIL; tail -20 gpurun_out/bench_default.log; exit 1; }
grep metric gpurun_out/bench_default.log
