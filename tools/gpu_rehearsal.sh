#!/bin/bash
# N-rank rehearsal of the driver's multi-GPU bench launch on ONE GPU: the exact torchrun form the
# driver uses (--nnodes=1 --nproc-per-node N --master-addr 127.0.0.1), gloo between the ranks
# (RCCL needs one GPU per rank), all N on the card, reduced resolution.  Exercises the env://
# rendezvous, the global-rank sampler, DDP + HIP SyncBN on its own group (early backward
# all-reduces), barriers, max-over-ranks timing and the rank-0-only JSON line.
# usage: tools/gpu_rehearsal.sh [N=2] [OUT=gpurun_out/rehearsal]
N=${1:-2}; OUT=${2:-gpurun_out/rehearsal}
mkdir -p "$OUT"
RTSEG_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29617 bench.py --gpus $N --steps 3 --warmup 2 --batch 2 \
  --height 256 --width 512 --no-infer > "$OUT/rehearsal_dp$N.log" 2>&1
rc=$?; grep -v alive "$OUT/rehearsal_dp$N.log" | tail -5; exit $rc
