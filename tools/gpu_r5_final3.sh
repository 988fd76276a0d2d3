#!/bin/bash
# Round-5 final check of the last tree: graft smoke(), the one-process GPU suite, the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5_final3
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -n 20 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
timeout -k 10 900 python3 -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1 || { tail -n 30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -n 20 $OUT/bench_default.err; exit 1; }
tail -n 1 $OUT/bench_default.json
