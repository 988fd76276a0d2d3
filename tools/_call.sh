set -o pipefail
mkdir -p gpurun_out/r6_stag
timeout -k 10 300 python -u -m pytest tests/test_conv_wres_gpu.py -k hreg -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_stag/tests.log 2>&1 || { tail -30 gpurun_out/r6_stag/tests.log; exit 1; }
tail -1 gpurun_out/r6_stag/tests.log
for i in 1 2; do timeout -k 10 200 python -u tools/bench_hreg.py > gpurun_out/r6_stag/bench_$i.txt 2>&1 || exit 1; done
