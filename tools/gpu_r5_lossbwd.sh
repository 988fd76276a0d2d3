#!/bin/bash
# Round 5: packed run form of the loss backward -- GPU tests, A/B microbench, PMC of both forms.
set -o pipefail
OUT=gpurun_out/r5_lossbwd
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "loss or ohem" > $OUT/pytest_loss.log 2>&1 || { tail -n 30 $OUT/pytest_loss.log; exit 1; }
tail -n 2 $OUT/pytest_loss.log
timeout -k 10 300 python -u tools/bench_loss_bwd.py --forms 0,1,2 > $OUT/bench.txt 2>&1 || { cat $OUT/bench.txt; exit 1; }
cat $OUT/bench.txt
cd /tmp && export TMPDIR=/tmp
for f in 1 2; do
  RTSEG_LOSS_BWD_RUN=$f timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY \
      -d $GRAFT_REPO_ROOT/$OUT/pmc_f$f -o pmc -- python3 $GRAFT_REPO_ROOT/tools/bench_loss_bwd.py --forms $f --reps 3 > $GRAFT_REPO_ROOT/$OUT/pmc_f$f.log 2>&1 || { tail -n 20 $GRAFT_REPO_ROOT/$OUT/pmc_f$f.log; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $GRAFT_REPO_ROOT/$OUT/pmc_f1 $GRAFT_REPO_ROOT/$OUT/pmc_f2 --filter seg_ce_bwd > $GRAFT_REPO_ROOT/$OUT/pmc_summary.txt || exit 1
rm -rf $GRAFT_REPO_ROOT/$OUT/pmc_f1 $GRAFT_REPO_ROOT/$OUT/pmc_f2
cat $GRAFT_REPO_ROOT/$OUT/pmc_summary.txt
echo done
