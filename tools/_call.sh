set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/r6_losshalf; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_determinism_gpu.py tests/test_ops_gpu.py -k "loss or seg or ohem" -v --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { grep -E "FAILED|^E  " $D/tests.log | head -30; tail -3 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for i in 1 2; do for v in 1 0; do
RTSEG_LOSS_HALF=$v timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-infer > $D/ab_${v}_$i.json 2> $D/ab.err || { tail -20 $D/ab.err; exit 1; }
echo "half=$v $(cut -c1-110 $D/ab_${v}_$i.json)"
done; done
