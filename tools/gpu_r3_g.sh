#!/bin/bash
# Round 3, call G: conv kernel tests on the new build (hw bf16 cvt, buffer gather), bench.py,
# then the guard-allocator probe with MIOpen off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3_g
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_igemm_gpu.py \
  tests/test_conv_gpu.py tests/test_conv_halo_gpu.py tests/test_bn_gpu.py tests/test_ops_gpu.py > gpurun_out/r3_g/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3_g/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_g/bench.json 2> gpurun_out/r3_g/bench.err
rc=$?
tail -1 gpurun_out/r3_g/bench.json | cut -c1-900
[ $rc -eq 0 ] || { tail -20 gpurun_out/r3_g/bench.err; exit $rc; }
bash tools/gpu_r3_d.sh
