set -o pipefail
mkdir -p gpurun_out/r6_c11
timeout -k 10 400 python -u -m pytest tests/test_ddp_model_gpu.py -x -v -s --timeout 600 --timeout-method thread -k two_ranks > gpurun_out/r6_c11/ddp.log 2>&1; rc=$?
grep -E "step-1 update|passed|failed" gpurun_out/r6_c11/ddp.log | tail -8
[ $rc -gt 1 ] && exit $rc
bash tools/gpu_zoo_latency.sh r6_zoo_latency espnet,regseg,fpenet
