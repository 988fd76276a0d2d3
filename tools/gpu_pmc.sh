#!/bin/bash
# PMC passes (one counter set per run) over conv kernels: MFMA busy vs waits vs issue
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM"
for kind in halo igemm; do
  for shape in 128,128,256,128 64,256,512,64; do
    i=0
    for P in "$P1" "$P2"; do
      i=$((i+1))
      timeout -s KILL 90 rocprofv3 --pmc $P -d $R/gpurun_out/pmc/${kind}_${shape//,/x}_p$i -o run -- python3 $R/tools/conv_probe.py --kind $kind --shape $shape --iters 10 > $R/gpurun_out/pmc/${kind}_${shape//,/x}_p$i.log 2>&1 || { echo "FAIL $kind $shape $i"; tail -5 $R/gpurun_out/pmc/${kind}_${shape//,/x}_p$i.log; exit 1; }
    done
  done
done
echo ok
