#!/bin/bash
# Round 5: fused-phase igemm data gradient of strided convs -- tests, microbench, bench A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5_dgradph
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_conv_gemm.py -x -q --timeout 120 \
    --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 300 python -u tools/bench_dgrad_phases.py > $OUT/micro.txt 2>&1 || { cat $OUT/micro.txt; exit 1; }
cat $OUT/micro.txt
RTSEG_CONV_DGRAD_PH=0 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_ph0.json 2> $OUT/bench_ph0.err || { tail -n 20 $OUT/bench_ph0.err; exit 1; }
tail -n 1 $OUT/bench_ph0.json
RTSEG_DECISIONS_OUT=$OUT/decisions_ph1.txt timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_ph1.json 2> $OUT/bench_ph1.err || { tail -n 20 $OUT/bench_ph1.err; exit 1; }
tail -n 1 $OUT/bench_ph1.json
RTSEG_CONV_DGRAD_PH=0 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_ph0b.json 2> $OUT/bench_ph0b.err || { tail -n 20 $OUT/bench_ph0b.err; exit 1; }
tail -n 1 $OUT/bench_ph0b.json
grep "dgrad" $OUT/decisions_ph1.txt | grep -E "\(2, 2\)|\(4, 4\)" || true
