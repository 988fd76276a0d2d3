#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probe_cfpnet.py cfpnet 6 > gpurun_out/probe_cfp.log 2>&1 || { echo PFAIL; tail -30 gpurun_out/probe_cfp.log; exit 1; }
grep seed gpurun_out/probe_cfp.log
RTSEG_POOL=0 timeout -k 10 200 python -u tools/probe_cfpnet.py cfpnet 6 > gpurun_out/probe_cfp2.log 2>&1 || { echo PFAIL2; tail -30 gpurun_out/probe_cfp2.log; exit 1; }
echo POOL0; grep seed gpurun_out/probe_cfp2.log
RTSEG_DISABLE_HIP=1 timeout -k 10 200 python -u tools/probe_cfpnet.py cfpnet 6 > gpurun_out/probe_cfp3.log 2>&1 || { echo PFAIL3; tail -30 gpurun_out/probe_cfp3.log; exit 1; }
echo NOHIP; grep seed gpurun_out/probe_cfp3.log
