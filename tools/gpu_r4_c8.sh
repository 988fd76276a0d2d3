#!/bin/bash
# round 4: headline bench with the round-4 conv kernels (fresh tuning DB -> gpurun_out), a second
# process on that DB, the steady-state kernel profile, the DDP / zoo re-checks, one batch-48 run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c8
mkdir -p $OUT
RTSEG_TUNE_DB=none RTSEG_TUNE_DB_OUT=$OUT/rtseg_conv_decisions.json RTSEG_DECISIONS_OUT=$OUT/decisions.txt \
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-700
RTSEG_TUNE_DB=$OUT/rtseg_conv_decisions.json timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-infer \
  > $OUT/bench_db.json 2> $OUT/bench_db.err || { tail -20 $OUT/bench_db.err; exit 1; }
tail -1 $OUT/bench_db.json | cut -c1-300
RTSEG_TUNE_DB=$OUT/rtseg_conv_decisions.json PROF_SKIP=8 PROF_PER_STEP=2 timeout -k 10 600 bash tools/profile_bench.sh $OUT --steps 6 --warmup 5 \
  > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
rm -f $OUT/trace.csv.gz
head -70 $OUT/steady.txt | cut -c1-180
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_ddp_model_gpu.py \
  "tests/test_zoo.py::test_zoo_hip_matches_torch_path_gpu[bisenetv2]" > $OUT/tests.log 2>&1
rc=$?; grep -E "amp=|passed|failed|train-BN" $OUT/tests.log; if [ $rc -gt 1 ]; then exit $rc; fi
RTSEG_TUNE_DB=$OUT/rtseg_conv_decisions.json RTSEG_STACK_DUMP=60 timeout -k 10 420 python -u bench.py --batch 48 --steps 10 --warmup 3 --no-infer \
  > $OUT/bench_b48.json 2> $OUT/bench_b48.err || { tail -40 $OUT/bench_b48.err; exit 1; }
tail -1 $OUT/bench_b48.json | cut -c1-300
