set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/r6_dappm; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_streams_gpu.py -v --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || { grep -E "FAILED|^E  " $D/tests.log | head -30; tail -3 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for i in 1 2; do for v in 1 0; do
RTSEG_BRANCH_STREAMS=$v timeout -k 10 180 python3 tools/profile_infer.py --iters 300 > $D/infer_${v}_$i.txt 2>&1 || { tail -5 $D/infer_${v}_$i.txt; exit 1; }
echo "streams=$v $(tail -1 $D/infer_${v}_$i.txt)"
done; done
