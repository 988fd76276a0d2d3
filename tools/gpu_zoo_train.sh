#!/bin/bash
mkdir -p gpurun_out
rm -f gpurun_out/zoo_train.jsonl
timeout -k 10 1100 python -u tools/zoo_train.py --batch 8 --steps 5 --warmup 3 --out gpurun_out/zoo_train.jsonl > gpurun_out/zoo_train.log 2>&1
rc=$?; grep -c images_per_s gpurun_out/zoo_train.jsonl; grep error gpurun_out/zoo_train.jsonl | head; exit $rc
