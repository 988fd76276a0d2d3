#!/bin/bash
# PMC of the stem kernels at DDRNet-23's stem geometry (batch 32, 1024 x 2048 -> 512 x 1024 x 64)
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5_stempmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM"
for kind in stem_nostore stem_apply stem_wgrad; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/${kind}_p$i -o run -- python3 $R/tools/conv_probe.py --kind $kind \
      --shape 3,1024,2048,64 --iters 5 > $OUT/${kind}_p$i.log 2>&1 || { echo "FAIL $kind $i"; tail -5 $OUT/${kind}_p$i.log; exit 1; }
  done
done
python3 $R/tools/pmc_summary.py $OUT/*_p? > $OUT/summary.txt || exit 1
rm -rf $OUT/*_p?
python3 $R/tools/pmc_table.py $OUT/summary.txt > $OUT/table.txt
echo ok
