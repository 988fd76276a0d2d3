#!/bin/bash
# 8-rank rehearsal of the driver's multi-GPU bench launch on ONE GPU: the exact
# torchrun form the driver uses (--nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1), gloo
# between the ranks (RCCL needs one GPU per rank), all 8 on the card, reduced resolution.
# Exercises: env:// rendezvous of 8 ranks, the global-rank sampler, DDP + HIP SyncBN on its own
# group (early backward all-reduces), barriers, max-over-ranks timing, rank-0-only JSON.
OUT=${1:-gpurun_out/rehearsal8}
mkdir -p "$OUT"
RTSEG_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29617 bench.py --gpus 8 --steps 3 --warmup 2 --batch 2 \
  --height 256 --width 512 --no-infer > "$OUT/rehearsal_dp8.log" 2>&1
rc=$?; grep -v alive "$OUT/rehearsal_dp8.log" | tail -5; exit $rc
