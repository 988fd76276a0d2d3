#!/bin/bash
# Round 5: the conv PMC table again on the final tree (16-byte epilogue stores / addend loads)
set -o pipefail
R=$GRAFT_REPO_ROOT
tools/gpu_pmc.sh gpurun_out/r5_pmc2 igemm+st:128,128,256,128 hreg_dg:128,128,256,128 whalo2:128,128,256,128 \
    igemm:64,256,512,64 igemm_dg:64,256,512,64 || exit 1
python3 $R/tools/pmc_table.py $R/gpurun_out/r5_pmc2/summary.txt > $R/gpurun_out/r5_pmc2/pmc_table.txt || exit 1
cat $R/gpurun_out/r5_pmc2/pmc_table.txt
