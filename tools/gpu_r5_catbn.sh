#!/bin/bash
# concat -> BN without the concat (ops.cat_bn_act): tests, CGNet / EDANet training A/B
OUT=${1:-gpurun_out/r5_catbn}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_concat_gpu.py \
  "tests/test_zoo.py::test_zoo_hip_matches_torch_path_gpu[cgnet]" "tests/test_zoo.py::test_zoo_hip_matches_torch_path_gpu[edanet]" \
  > "$OUT/tests.log" 2>&1 || exit $?
for v in 1 0; do
  RTSEG_CONCAT_SINK=$v timeout -k 10 400 python3 -u tools/zoo_train.py --models cgnet,edanet --batch 8 --steps 10 \
    --warmup 3 --out "$OUT/zoo_train_sink$v.jsonl" > "$OUT/zoo_train_sink$v.log" 2>&1 || exit $?
done
