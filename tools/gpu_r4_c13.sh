#!/bin/bash
# round 4: whalo immediate-offset K loop (tests + A/B vs the round-4 numbers), steady-state
# profiles of the slowest zoo models per parameter (verdict item 7)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r4_c13
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_wres_gpu.py -k whalo > $OUT/whalo_tests.log 2>&1 || { tail -30 $OUT/whalo_tests.log; exit 1; }
tail -1 $OUT/whalo_tests.log
timeout -k 10 300 python -u tools/bench_conv.py --shapes 2,4,6 --only wgrad > $OUT/bench_whalo.txt 2>&1 || { tail -20 $OUT/bench_whalo.txt; exit 1; }
grep -E "shape|whalo|wgrad" $OUT/bench_whalo.txt
bash tools/gpu_pmc.sh $OUT/pmc whalo:64,256,512,64 whalo:128,128,256,128 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
for m in aglnet lednet fddwnet contextnet; do
  PROF_SKIP=5 PROF_PER_STEP=1 timeout -k 10 280 bash tools/profile_bench.sh $OUT/$m --model $m --batch 8 --steps 3 --warmup 4 \
    > $OUT/$m.log 2>&1 || { tail -20 $OUT/$m.log; exit 1; }
  rm -f $OUT/$m/trace.csv.gz $OUT/$m/kernel_stats.csv
  echo "== $m"; head -24 $OUT/$m/steady.txt | cut -c1-170
done
