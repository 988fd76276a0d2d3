#!/bin/bash
# round-end style verification (new-kernel tests, GPU suite, smoke, bench) + rocprofv3 steady profile
mkdir -p gpurun_out
bash tools/gpu_verify2.sh || exit 1
PROF_SKIP=4 bash tools/profile_bench.sh gpurun_out/prof_final --steps 6 --warmup 4 || exit 1
head -12 gpurun_out/prof_final/steady.txt
