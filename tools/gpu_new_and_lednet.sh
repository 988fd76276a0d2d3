#!/bin/bash
# New kernel tests (augment / act / shuffle), then the LEDNet zoo case serialised to locate a fault.
mkdir -p gpurun_out
fault() { grep -qE "illegal memory access|hipError|Memory access fault|Aborted|core dumped" "$1"; }
timeout -k 10 400 python -u -m pytest tests/test_augment_gpu.py tests/test_act_gpu.py tests/test_shuffle_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/n_new.log 2>&1
rc=$?; tail -5 gpurun_out/n_new.log
if [ $rc -gt 1 ] || fault gpurun_out/n_new.log; then echo "STOP rc=$rc"; exit 1; fi
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest "tests/test_zoo.py::test_zoo_hip_matches_torch_path_gpu[lednet]" -x -q --timeout 240 --timeout-method thread > gpurun_out/n_lednet.log 2>&1
rc=$?; grep -nE "Error|error|rtseg|ops\.|passed|failed" gpurun_out/n_lednet.log | head -40
exit 0
