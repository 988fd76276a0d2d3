#!/bin/bash
# Round 5: L2 (TCC) hit rate and memory-side read requests of the heaviest conv kernels, one
# rocprofv3 --pmc pass per probe (4 TCC counters: the per-block limit).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5_l2pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_WAVES SQ_BUSY_CYCLES"
for spec in igemm+st:128,128,256,128 whalo2:128,128,256,128 hreg_dg:128,128,256,128 igemm+st:256,64,128,256 whalo:64,256,512,64; do
  kind=${spec%%:*}; shape=${spec#*:}
  extra=""
  if [[ $kind == *+st ]]; then kind=${kind%+st}; extra="--stats"; fi
  tag=${spec//[:,+]/_}
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/${tag}_p1 -o run -- python3 $R/tools/conv_probe.py --kind $kind --shape $shape --iters 10 $extra > $OUT/${tag}_p1.log 2>&1 || { echo "FAIL $spec"; tail -5 $OUT/${tag}_p1.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT/*_p1 --filter rtseg > $OUT/summary.txt || exit 1
rm -rf $OUT/*_p1
cat $OUT/summary.txt
cd $R
RTSEG_PROBE_OPS=$OUT/step_ops.txt timeout -k 10 400 python -u bench.py --steps 2 --warmup 2 > $OUT/probe_bench.log 2>&1 || { tail -n 20 $OUT/probe_bench.log; exit 1; }
cat $OUT/step_ops.txt
