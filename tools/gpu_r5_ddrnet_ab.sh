#!/bin/bash
# Bisection of the DDRNet train-BN numerics (test_zoo ddrnet case): test order and kernel families
OUT=${1:-gpurun_out/r5_ab}
mkdir -p "$OUT"
T='tests/test_zoo.py::test_zoo_hip_matches_torch_path_gpu[ddrnet]'
run() { local tag=$1; shift; timeout -k 10 300 python3 -u -m pytest "$@" -q -s -p no:cacheprovider > "$OUT/$tag.log" 2>&1; grep -h "train-BN:" "$OUT/$tag.log" | sed "s/^/$tag: /"; }
run prefix tests/test_bn_gpu.py tests/test_syncbn_gpu.py "$T"
RTSEG_HIP_OFF=bn run off_bn "$T"
RTSEG_HIP_OFF=interp run off_interp "$T"
RTSEG_HIP_OFF=loss run off_loss "$T"
RTSEG_HIP_OFF=pool run off_pool "$T"
exit 0
