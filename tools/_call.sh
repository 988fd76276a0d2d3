set -o pipefail
D=gpurun_out/r6_tol; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_conv_stem_gpu.py tests/test_zoo.py tests/test_routed_conv_gpu.py -v --timeout 200 --timeout-method thread > $D/tests2.log 2>&1; rc=$?
grep -E "passed|failed" $D/tests2.log | tail -3
grep -E "^FAILED|Greatest" $D/tests2.log | head -40
exit $rc
