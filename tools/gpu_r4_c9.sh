#!/bin/bash
# round 4: hreg 4-wave variant + concat sink (tests, A/B), headline bench on a fresh tuning DB,
# STDC2 + detail b16 profile with / without the concat sink, DDP rehearsal (CE)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c9
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_wres_gpu.py tests/test_concat_gpu.py -k "hreg or concat or stdc" > $OUT/kernel_tests.log 2>&1 || { tail -40 $OUT/kernel_tests.log; exit 1; }
tail -2 $OUT/kernel_tests.log
timeout -k 10 300 python -u tools/bench_conv.py --shapes 2,4,6 --only fwd,dgrad > $OUT/bench_hreg2.txt 2>&1 || { tail -20 $OUT/bench_hreg2.txt; exit 1; }
grep hreg $OUT/bench_hreg2.txt
RTSEG_TUNE_DB=none RTSEG_TUNE_DB_OUT=$OUT/rtseg_conv_decisions.json RTSEG_DECISIONS_OUT=$OUT/decisions.txt \
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-1200
for s in 0 1; do
  RTSEG_CONCAT_SINK=$s timeout -k 10 300 python -u bench.py --model stdc --arch stdc2 --detail-head --batch 16 --steps 10 --warmup 5 --no-infer \
    > $OUT/stdc_sink$s.json 2> $OUT/stdc_sink$s.err || { tail -20 $OUT/stdc_sink$s.err; exit 1; }
  tail -1 $OUT/stdc_sink$s.json | cut -c1-300
done
PROF_SKIP=8 PROF_PER_STEP=2 timeout -k 10 500 bash tools/profile_bench.sh $OUT/stdc --model stdc --arch stdc2 --detail-head --batch 16 --steps 6 --warmup 5 \
  > $OUT/stdc_prof.log 2>&1 || { tail -20 $OUT/stdc_prof.log; exit 1; }
rm -f $OUT/stdc/trace.csv.gz
head -40 $OUT/stdc/steady.txt | cut -c1-160
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_ddp_model_gpu.py > $OUT/ddp.log 2>&1
rc=$?; grep -E "amp=|passed|failed" $OUT/ddp.log | cut -c1-400; exit $rc
