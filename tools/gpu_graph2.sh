#!/bin/bash
# graph step on the launch-gap-heavy models (BiSeNetV2, STDC2+detail at batch 16) + a tuning
# database collected over all runs (DDRNet-23 b32 first: the headline config)
mkdir -p gpurun_out
export RTSEG_TUNE_DB=gpurun_out/rtseg_conv_decisions.json RTSEG_TUNE_DB_OUT=gpurun_out/rtseg_conv_decisions.json
run() {
  local tag=$1; shift
  timeout -k 10 420 python -u bench.py --steps 10 --warmup 5 --no-infer "$@" > gpurun_out/h_$tag.json 2> gpurun_out/h_$tag.err || { tail -20 gpurun_out/h_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.load(open('gpurun_out/h_$tag.json'));print(d['value'],d['ms_per_step'])")"
}
run ddr32 --batch 32
run bise16_eager --model bisenetv2 --batch 16
run bise16_graph --model bisenetv2 --batch 16 --graph-step
run stdc16_eager --model stdc --arch stdc2 --detail-head --batch 16
run stdc16_graph --model stdc --arch stdc2 --detail-head --batch 16 --graph-step
