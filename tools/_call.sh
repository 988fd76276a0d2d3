set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/r6_dwmult_fps; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_dwconv_gpu.py -v --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { grep -E "FAILED|^E  " $D/tests.log | head -30; tail -3 $D/tests.log; exit 1; }
tail -2 $D/tests.log
timeout -k 10 500 python -u tools/zoo_fps.py --only bisenetv2,ddrnet,stdc,espnetv2,fastscnn,dfanet --out $D/fps.jsonl > $D/fps.log 2>&1 || { tail -5 $D/fps.log; exit 1; }
cut -c1-200 $D/fps.jsonl
