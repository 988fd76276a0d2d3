#!/bin/bash
# one GPU call: the new-kernel tests, smoke(), the headline bench with the new paths on and off,
# then the whole one-process GPU suite (a crash stops the call; a failing new-kernel NUMERICS
# test keeps the new paths off for the benches)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/${FINAL_OUT:-final}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv_stem_gpu.py -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/stem.log 2>&1
rc=$?
tail -4 $OUT/stem.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
NEW="RTSEG_CONV_STEM=1 RTSEG_TWIN_CONV=1"
if [ $rc -eq 1 ]; then NEW="RTSEG_CONV_STEM=0 RTSEG_TWIN_CONV=0"; echo "new paths OFF"; fi
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
env $NEW RTSEG_DECISIONS_OUT=$OUT/decisions.txt timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 \
  > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-400
RTSEG_CONV_STEM=0 RTSEG_TWIN_CONV=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-infer \
  > $OUT/bench_off.json 2> $OUT/bench_off.err || { tail -20 $OUT/bench_off.err; exit 1; }
tail -1 $OUT/bench_off.json | cut -c1-300
[ -n "$SKIP_SUITE" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -6 $OUT/pytest_gpu.log
exit $rc
