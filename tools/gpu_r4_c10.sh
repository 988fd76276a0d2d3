#!/bin/bash
# round 4: STDC2 + detail b16 profile (concat-elimination "before"), the whole zoo's HIP-vs-fp64
# numerics (36 models, frozen + train BN, bf16 production path), one batch-48 headline run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c10
mkdir -p $OUT
PROF_SKIP=8 PROF_PER_STEP=2 timeout -k 10 500 bash tools/profile_bench.sh $OUT/stdc --model stdc --arch stdc2 --detail-head --batch 16 --steps 6 --warmup 5 \
  > $OUT/stdc_prof.log 2>&1 || { tail -20 $OUT/stdc_prof.log; exit 1; }
rm -f $OUT/stdc/trace.csv.gz
grep -m1 metric $OUT/stdc/bench.log | cut -c1-300
head -40 $OUT/stdc/steady.txt | cut -c1-160
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_zoo.py -k zoo_hip_matches > $OUT/zoo.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $OUT/zoo.log | tail -5; if [ $rc -gt 1 ]; then exit $rc; fi
RTSEG_STACK_DUMP=60 timeout -k 10 600 python -u bench.py --batch 48 --steps 10 --warmup 3 --no-infer \
  > $OUT/bench_b48.json 2> $OUT/bench_b48.err || { grep -v "^  File\|^Thread" $OUT/bench_b48.err | tail -20; exit 1; }
tail -1 $OUT/bench_b48.json | cut -c1-400
