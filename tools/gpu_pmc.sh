#!/bin/bash
# PMC passes (one counter set per run) over conv kernels: MFMA busy vs waits vs issue.
# usage: tools/gpu_pmc.sh OUTDIR kind:cin,h,w,cout [...]   (kinds: tools/conv_probe.py --kind)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM"
for spec in "$@"; do
  kind=${spec%%:*}; shape=${spec#*:}
  extra=""
  if [[ $kind == *+st ]]; then kind=${kind%+st}; extra="--stats"; fi
  tag=${spec//[:,+]/_}
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/${tag}_p$i -o run -- python3 $R/tools/conv_probe.py --kind $kind --shape $shape --iters 10 $extra > $OUT/${tag}_p$i.log 2>&1 || { echo "FAIL $spec pass $i"; tail -5 $OUT/${tag}_p$i.log; exit 1; }
  done
done
python3 $R/tools/pmc_summary.py $OUT/*_p? > $OUT/summary.txt || exit 1
# raw rocprofv3 databases are large (gpurun copies back <= 64 MiB): keep the summary only
rm -rf $OUT/*_p?
echo ok
