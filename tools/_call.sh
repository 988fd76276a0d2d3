set -o pipefail
mkdir -p gpurun_out/r6_dw
timeout -k 10 400 python -u -m pytest tests/test_dwconv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_dw/tests.log 2>&1 || { tail -30 gpurun_out/r6_dw/tests.log; exit 1; }
tail -1 gpurun_out/r6_dw/tests.log
RTSEG_DW_CS=0 timeout -k 10 200 python -u tools/bench_dw.py > gpurun_out/r6_dw/bench_base.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_dw.py > gpurun_out/r6_dw/bench_cs.txt 2>&1 || exit 1
cat gpurun_out/r6_dw/bench_base.txt gpurun_out/r6_dw/bench_cs.txt | grep -v amdgpu
timeout -k 10 600 python -u -m pytest tests/test_syncbn_collectives_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_dw/coll.log 2>&1; tail -3 gpurun_out/r6_dw/coll.log
