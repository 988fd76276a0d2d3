#!/bin/bash
# Round-5 closing evidence (2): the one-process GPU suite, an A/B of the headline against the
# previous build (RTSEG_LIB_PATH=_C/librtseg_hip_prev.so: before the 16-byte hreg/wres/halo
# stores), the default bench and a steady-state profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5_closing2
PREV=$R/realtime_semantic_segmentation_pytorch_amd/_C/librtseg_hip_prev.so
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1 || { tail -n 30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
RTSEG_LIB_PATH=$PREV timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench_prev.json 2> $OUT/bench_prev.err || { tail -n 20 $OUT/bench_prev.err; exit 1; }
tail -n 1 $OUT/bench_prev.json
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench_new.json 2> $OUT/bench_new.err || { tail -n 20 $OUT/bench_new.err; exit 1; }
tail -n 1 $OUT/bench_new.json
timeout -k 10 300 python3 -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -n 20 $OUT/bench_default.err; exit 1; }
tail -n 1 $OUT/bench_default.json
tools/profile_bench.sh gpurun_out/r5_closing2/prof --steps 6 --warmup 3 > $OUT/prof.log 2>&1 || { tail -n 20 $OUT/prof.log; exit 1; }
echo closing-done
