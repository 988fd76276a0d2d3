#!/bin/bash
# Round 3, call E: buffer-resource gather in conv_igemm -- kernel tests, per-shape bench, bench.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3_e
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_igemm_gpu.py \
  tests/test_conv_gpu.py tests/test_deconv_unpool_gpu.py tests/test_conv_halo_gpu.py > gpurun_out/r3_e/tests.log 2>&1
rc=$?
tail -5 gpurun_out/r3_e/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_conv.py --batch 32 --only fwd,dgrad > gpurun_out/r3_e/bench_conv.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r3_e/bench_conv.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_e/bench.json 2> gpurun_out/r3_e/bench.err
rc=$?
tail -2 gpurun_out/r3_e/bench.json | cut -c1-600
exit $rc
