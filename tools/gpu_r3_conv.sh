#!/bin/bash
# conv kernel numerics tests, then the per-shape conv bench (CONV_ONLY passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r3_conv
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_igemm_gpu.py \
  tests/test_conv_halo_gpu.py ${CONV_TESTS:-} > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/bench_conv.py --only ${CONV_ONLY:-fwd,dgrad} > $OUT/bench_conv.txt 2>&1 || { tail -20 $OUT/bench_conv.txt; exit 1; }
cut -c1-160 $OUT/bench_conv.txt
