set -o pipefail
bash tools/gpu_pmc.sh gpurun_out/r6_pmc hreg4+st:128,128,256,128 hreg4_dg:128,128,256,128 whalo2:128,128,256,128 igemm+st:256,64,128,256 wres+st:64,256,512,64 || exit 1
python3 tools/pmc_table.py gpurun_out/r6_pmc/summary.txt > gpurun_out/r6_pmc/pmc_table.txt 2>&1 || true
cat gpurun_out/r6_pmc/pmc_table.txt | head -30
