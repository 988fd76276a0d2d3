#!/bin/bash
# Round 3, call F: flat vs buffer gather in conv_igemm (RTSEG_IGEMM_GATHER=0|1): per-shape time and PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3_f
export PYTHONUNBUFFERED=1
for g in 0 1; do
  RTSEG_IGEMM_GATHER=$g timeout -k 10 200 python -u tools/bench_conv.py --batch 32 --only fwd,dgrad --shapes 0,2,4,6 \
    > gpurun_out/r3_f/bench_conv_g$g.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r3_f/bench_conv_g$g.txt | grep -v halo
done
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM"
for g in 0 1; do
  for shape in 64,256,512,64 128,128,256,128; do
    i=0
    for P in "$P1" "$P2"; do
      i=$((i+1))
      out=$R/gpurun_out/r3_f/pmc_g${g}_${shape//,/x}_p$i
      RTSEG_IGEMM_GATHER=$g timeout -s KILL 90 rocprofv3 --pmc $P -d $out -o run -- python3 $R/tools/conv_probe.py --kind igemm --shape $shape --iters 10 > $out.log 2>&1 || { echo "FAIL $g $shape $i"; tail -5 $out.log; exit 1; }
    done
  done
done
cd $R && python3 tools/pmc_summary.py gpurun_out/r3_f > gpurun_out/r3_f/pmc_summary.txt 2>&1; tail -80 gpurun_out/r3_f/pmc_summary.txt
