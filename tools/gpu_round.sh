#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
RTSEG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --batch 4 --no-infer > gpurun_out/b_gloo2.log 2>&1 || { echo GLOOFAIL; tail -40 gpurun_out/b_gloo2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b_gloo2.log | tail -3
