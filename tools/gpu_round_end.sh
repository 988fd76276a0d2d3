#!/bin/bash
# twin-node tests, the headline bench, a profile without weight shadows (fused-optimizer A/B),
# then the other BASELINE-config benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/end
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_conv_stem_gpu.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/stem.log 2>&1 || { tail -20 $OUT/stem.log; exit 1; }
tail -1 $OUT/stem.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-300
RTSEG_WEIGHT_SHADOW=0 PROF_OUT=end/prof_noshadow bash tools/gpu_prof.sh | grep -E "steps analysed|fused_opt|CUDAFunctor_add|copy" || exit 1
MODELS_OUT=end bash tools/gpu_models.sh
