#!/bin/bash
# Zoo training throughput (bf16, batch 8, 1024x2048) for TRAIN_MODELS and inference FPS (batch 1,
# 1024x512, fp32 and bf16) for FPS_MODELS, appended to gpurun_out/zoo/*_TAG.jsonl (one GPU call per
# chunk; either list may be "-" for none).
# usage: tools/gpu_zoo_sweep.sh TAG TRAIN_MODELS FPS_MODELS
TAG=$1; TRAIN=$2; FPS=${3:--}
mkdir -p gpurun_out/zoo
if [ "$TRAIN" != "-" ]; then
  timeout -k 10 ${TRAIN_TIMEOUT:-560} python -u tools/zoo_train.py --batch 8 --steps 5 --warmup 3 --models $TRAIN --out gpurun_out/zoo/train_$TAG.jsonl > gpurun_out/zoo/train_$TAG.log 2>&1
  rc=$?; echo "train rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
fi
if [ "$FPS" != "-" ]; then
  timeout -k 10 500 python -u tools/zoo_fps.py --only $FPS --out gpurun_out/zoo/fps_$TAG.jsonl > gpurun_out/zoo/fps_$TAG.log 2>&1
  rc=$?; echo "fps rc=$rc"; exit $rc
fi
