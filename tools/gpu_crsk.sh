#!/bin/bash
# fused-optimizer tests (shadow layouts), the headline bench, and its steady-state profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/crsk
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_fused_optim_gpu.py tests/test_conv_stem_gpu.py -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { grep -E "^E |FAILED" $OUT/tests.log | head; tail -3 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-300
PROF_OUT=crsk/prof bash tools/gpu_prof.sh | grep -E "steps analysed|fused_opt|shadow_crsk|CUDAFunctor_add|stem_" || exit 1
