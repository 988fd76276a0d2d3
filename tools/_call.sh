set -o pipefail
mkdir -p gpurun_out/r6_kd2
timeout -k 10 300 python -u -m pytest tests/test_conv_stem7_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_kd2/tests.log 2>&1 || { tail -30 gpurun_out/r6_kd2/tests.log; exit 1; }
tail -1 gpurun_out/r6_kd2/tests.log
timeout -k 10 200 python -u tools/bench_stem7.py > gpurun_out/r6_kd2/stem7.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r6_kd2/stem7.txt
timeout -k 10 500 python -u bench.py --kd --batch 16 --steps 10 --warmup 4 --no-infer > gpurun_out/r6_kd2/bench_kd_b16.json 2> gpurun_out/r6_kd2/bench_kd.err || { tail -20 gpurun_out/r6_kd2/bench_kd.err; exit 1; }
tail -1 gpurun_out/r6_kd2/bench_kd_b16.json | cut -c1-200
