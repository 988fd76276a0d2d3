#!/bin/bash
# BiSeNetV2 bf16-vs-fp32 gradient check at two earlier commits (worktrees under _bisect/) and on the
# current tree, then the kernel tests touched this round, the BN bandwidth bench, three zoo models.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
OUT=$GRAFT_REPO_ROOT/gpurun_out/bisect
mkdir -p $OUT
T="tests/test_train_numerics_gpu.py::test_bf16_step_vs_fp32_reference[bisenetv2_aux]"
for w in _bisect/a _bisect/b .; do
  tag=$(basename $w)
  (cd $w && timeout -k 10 200 python -u -m pytest -x -q -s --timeout 180 --timeout-method thread "$T" > $OUT/bis_$tag.log 2>&1)
  echo "$w rc=$?"; grep -E "cos median" $OUT/bis_$tag.log
done
rm -rf _bisect
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_act_gpu.py tests/test_bn_gpu.py \
  tests/test_deconv_unpool_gpu.py tests/test_dwconv_gpu.py tests/test_routed_conv_gpu.py $TAPTEST > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; grep -E "^FAILED" $OUT/tests.log | head; [ $rc -eq 0 ] || exit 1
timeout -k 10 150 python -u tools/bench_bn_bw.py > $OUT/bw.txt 2>&1 && tail -5 $OUT/bw.txt
timeout -k 10 400 python -u tools/zoo_train.py --batch 8 --steps 5 --warmup 3 --models cfpnet,canet,adscnet --out $OUT/zoo.jsonl > $OUT/zoo.log 2>&1
cut -c1-150 $OUT/zoo.jsonl
