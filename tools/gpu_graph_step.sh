#!/bin/bash
# graph-captured training step: numerics vs eager, then eager vs graph at small and large batch
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_graph_step_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/g_test.log 2>&1 || { tail -40 gpurun_out/g_test.log; exit 1; }
tail -1 gpurun_out/g_test.log
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --no-infer "$@" > gpurun_out/g_$tag.json 2> gpurun_out/g_$tag.err || { tail -20 gpurun_out/g_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.load(open('gpurun_out/g_$tag.json'));print(d['value'],d['ms_per_step'])")"
}
run cgnet8_eager --model cgnet --batch 8
run cgnet8_graph --model cgnet --batch 8 --graph-step
run ddr32_graph --batch 32 --graph-step
