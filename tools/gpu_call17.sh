#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/bench_conv.py --only dgrad,dgrad_bn --shapes 0,2,4,6,7,9 --cfgs 1,2,4 > gpurun_out/bench_conv_dgbn.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bench_conv_dgbn.log; exit $rc
