#!/bin/bash
# KD teacher graph test + KD bench (graph vs eager teacher) + CGNet (PReLU-heavy) training bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kd_teacher_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/k_test.log 2>&1 || { tail -30 gpurun_out/k_test.log; exit 1; }
tail -1 gpurun_out/k_test.log
timeout -k 10 400 python -u bench.py --kd --batch 16 --steps 10 --warmup 4 --no-infer > gpurun_out/k_bench_graph.json 2> gpurun_out/k_bench_graph.err || { tail -20 gpurun_out/k_bench_graph.err; exit 1; }
cat gpurun_out/k_bench_graph.json
RTSEG_KD_EAGER=1 timeout -k 10 400 python -u bench.py --kd --batch 16 --steps 10 --warmup 4 --no-infer > gpurun_out/k_bench_eager.json 2> gpurun_out/k_bench_eager.err || { tail -20 gpurun_out/k_bench_eager.err; exit 1; }
cat gpurun_out/k_bench_eager.json
timeout -k 10 300 python -u bench.py --model cgnet --batch 16 --steps 10 --warmup 4 --no-infer > gpurun_out/k_cgnet.json 2> gpurun_out/k_cgnet.err || { tail -20 gpurun_out/k_cgnet.err; exit 1; }
cat gpurun_out/k_cgnet.json
RTSEG_DISABLE_ACT=1 timeout -k 10 300 python -u bench.py --model cgnet --batch 16 --steps 10 --warmup 4 --no-infer > gpurun_out/k_cgnet_noact.json 2> gpurun_out/k_cgnet_noact.err || { tail -20 gpurun_out/k_cgnet_noact.err; exit 1; }
cat gpurun_out/k_cgnet_noact.json
