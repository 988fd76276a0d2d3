#!/bin/bash
# Round 5: 16-byte residual / addend loads in the igemm epilogue -- tests, then an A/B of the
# headline against the previous build (RTSEG_LIB_PATH=_C/librtseg_hip_prev.so), interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5_sideload
PREV=$R/realtime_semantic_segmentation_pytorch_amd/_C/librtseg_hip_prev.so
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_conv_halo_gpu.py tests/test_conv_wres_gpu.py tests/test_conv_igemm_gpu.py \
    tests/test_routed_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
for i in 1 2; do
  RTSEG_LIB_PATH=$PREV timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_prev$i.json 2> $OUT/bench_prev$i.err || { tail -n 20 $OUT/bench_prev$i.err; exit 1; }
  tail -n 1 $OUT/bench_prev$i.json
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_new$i.json 2> $OUT/bench_new$i.err || { tail -n 20 $OUT/bench_new$i.err; exit 1; }
  tail -n 1 $OUT/bench_new$i.json
done
