#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_misc_ops_gpu.py > gpurun_out/t_misc.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_misc.log; exit 1; }
tail -2 gpurun_out/t_misc.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 5 --batch 16 --kd --no-infer > gpurun_out/b_kd.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/b_kd.log; exit 1; }
tail -1 gpurun_out/b_kd.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_kd16b -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --batch 16 --kd --no-infer > $GRAFT_REPO_ROOT/gpurun_out/p_kd.log 2>&1 || { echo PROFFAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/p_kd.log; exit 1; }
echo done
