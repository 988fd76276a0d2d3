#!/bin/bash
# round 4: new halo kernels (tests, A/B bench, PMC), zoo bf16 calibration subset, DDP + convergence
mkdir -p gpurun_out/r4_c7
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_wres_gpu.py > gpurun_out/r4_c7/kernel_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_conv.py --shapes 2,4,6 --only fwd,dgrad > gpurun_out/r4_c7/bench_hreg.txt 2>&1 || exit $?
bash tools/gpu_pmc.sh gpurun_out/r4_c7/pmc wres:64,256,512,64 wres+st:64,256,512,64 whalo:64,256,512,64 hreg:128,128,256,128 hreg_dg:128,128,256,128 > gpurun_out/r4_c7/pmc.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_zoo.py -k "zoo_hip_matches and (ddrnet or bisenetv2 or stdc or cgnet or enet or lednet or fastscnn or segnet)" > gpurun_out/r4_c7/zoo.log 2>&1
rc=$?; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest -v -s --durations=0 --timeout 400 --timeout-method thread -m gpu tests/test_ddp_model_gpu.py tests/test_convergence.py -k "converges or ddp" > gpurun_out/r4_c7/pytest.log 2>&1
