set -o pipefail
mkdir -p gpurun_out/r6_stage
timeout -k 10 300 python -u -m pytest tests/test_conv_wres_gpu.py -k hreg -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_stage/tests.log 2>&1 || { tail -30 gpurun_out/r6_stage/tests.log; exit 1; }
tail -1 gpurun_out/r6_stage/tests.log
timeout -k 10 200 python -u tools/bench_hreg.py > gpurun_out/r6_stage/bench.txt 2>&1 || exit 1
for i in 1 2; do
  for h in 0 1; do
    RTSEG_CONV_HREG4=$h timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-infer > gpurun_out/r6_stage/b_h${h}_$i.json 2> gpurun_out/r6_stage/b_h${h}_$i.err || exit 1
    tail -1 gpurun_out/r6_stage/b_h${h}_$i.json | cut -c1-120
  done
done
timeout -k 10 600 python -u -m pytest tests/test_syncbn_collectives_gpu.py tests/test_ddp_model_gpu.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r6_stage/ddp.log 2>&1 || { tail -30 gpurun_out/r6_stage/ddp.log; exit 1; }
grep -E "rel|passed|failed" gpurun_out/r6_stage/ddp.log | tail -12
