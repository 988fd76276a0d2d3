#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench path on ONE GPU (gloo between the ranks, both on the
# card): torchrun env:// rendezvous, DDP + HIP SyncBN on its own group, max-over-ranks timing, JSON
mkdir -p gpurun_out
RTSEG_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 3 --warmup 2 --batch 4 --no-infer \
  > gpurun_out/rehearsal_dp2.log 2>&1
rc=$?; grep -v alive gpurun_out/rehearsal_dp2.log | tail -5; exit $rc
