#!/bin/bash
# Round 5: 16-byte igemm epilogue stores -- tests, microbench, bench A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5_wide
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_conv_gemm.py tests/test_routed_conv_gpu.py -x -q \
    --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 300 python -u tools/bench_igemm_wide.py > $OUT/micro.txt 2>&1 || { cat $OUT/micro.txt; exit 1; }
cat $OUT/micro.txt
RTSEG_IGEMM_WIDE_STORE=0 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_w0.json 2> $OUT/bench_w0.err || { tail -n 20 $OUT/bench_w0.err; exit 1; }
tail -n 1 $OUT/bench_w0.json
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_w1.json 2> $OUT/bench_w1.err || { tail -n 20 $OUT/bench_w1.err; exit 1; }
tail -n 1 $OUT/bench_w1.json
RTSEG_IGEMM_WIDE_STORE=0 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_w0b.json 2> $OUT/bench_w0b.err || { tail -n 20 $OUT/bench_w0b.err; exit 1; }
tail -n 1 $OUT/bench_w0b.json
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_w1b.json 2> $OUT/bench_w1b.err || { tail -n 20 $OUT/bench_w1b.err; exit 1; }
tail -n 1 $OUT/bench_w1b.json
