#!/bin/bash
# per-GPU batch sweep of the headline bench, then the default bench + rocprofv3 steady profile
mkdir -p gpurun_out
for b in 48 64; do
  timeout -k 10 400 python -u bench.py --batch $b --steps 10 --warmup 4 --no-infer > gpurun_out/f_bench_b$b.json 2> gpurun_out/f_bench_b$b.err || { tail -20 gpurun_out/f_bench_b$b.err; exit 1; }
  cat gpurun_out/f_bench_b$b.json
done
bash tools/gpu_bench.sh b32
