#!/bin/bash
# 1-GPU headline bench + a rocprofv3 steady-state profile of the same step (one GPU call).
# usage: tools/gpu_bench.sh TAG [bench args...]
TAG=${1:-b32}; shift || true
mkdir -p gpurun_out
RTSEG_DECISIONS_OUT=gpurun_out/decisions_$TAG.txt timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
tail -3 gpurun_out/bench_$TAG.err; cat gpurun_out/bench_$TAG.json
if [ $rc -ne 0 ]; then exit $rc; fi
PROF_SKIP=${PROF_SKIP:-4} bash tools/profile_bench.sh gpurun_out/prof_$TAG --steps 6 --warmup 4 "$@"
rc=$?
head -12 gpurun_out/prof_$TAG/steady.txt
exit $rc
