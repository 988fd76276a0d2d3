#!/bin/bash
# round 4: STDC2 + detail b16 steady profiles with / without the concat sink, the 2-rank STDC
# mismatch bisected by kernel family, the whole zoo's HIP-vs-fp64 numerics (36 models)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c10
mkdir -p $OUT
for s in 1 0; do
  RTSEG_CONCAT_SINK=$s PROF_SKIP=8 PROF_PER_STEP=1 timeout -k 10 400 bash tools/profile_bench.sh $OUT/stdc_sink$s --model stdc --arch stdc2 --detail-head --batch 16 --steps 6 --warmup 5 \
    > $OUT/stdc_prof$s.log 2>&1 || { tail -20 $OUT/stdc_prof$s.log; exit 1; }
  rm -f $OUT/stdc_sink$s/trace.csv.gz
  head -12 $OUT/stdc_sink$s/steady.txt
done
timeout -k 10 500 python -u tools/probe_ddp_bisect.py --model stdc2_aux --families ",bn,pool,gate,interp,loss" > $OUT/ddp_bisect.log 2>&1 || { tail -30 $OUT/ddp_bisect.log; exit 1; }
grep -v "^\s*$" $OUT/ddp_bisect.log | grep -v amdgpu | head -80
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_zoo.py -k zoo_hip_matches > $OUT/zoo.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $OUT/zoo.log | tail -8; exit $rc
