#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/last_bench.json 2> gpurun_out/last_bench.err || { tail -20 gpurun_out/last_bench.err; exit 1; }
cat gpurun_out/last_bench.json
