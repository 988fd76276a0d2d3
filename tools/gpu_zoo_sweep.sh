#!/bin/bash
# Zoo training throughput (bf16, batch 8, 1024x2048) + inference FPS (batch 1, 1024x512, fp32 and bf16)
# for a comma list of models, appended to gpurun_out/zoo/*.jsonl (one GPU call per chunk).
# usage: tools/gpu_zoo_sweep.sh TAG model1,model2,...
TAG=$1; MODELS=$2
mkdir -p gpurun_out/zoo
timeout -k 10 560 python -u tools/zoo_train.py --batch 8 --steps 5 --warmup 3 --models $MODELS --out gpurun_out/zoo/train_$TAG.jsonl > gpurun_out/zoo/train_$TAG.log 2>&1
rc=$?; echo "train rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 500 python -u tools/zoo_fps.py --only $MODELS --out gpurun_out/zoo/fps_$TAG.jsonl > gpurun_out/zoo/fps_$TAG.log 2>&1
rc=$?; echo "fps rc=$rc"; exit $rc
