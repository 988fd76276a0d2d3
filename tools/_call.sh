set -o pipefail
mkdir -p gpurun_out/r6_kd3
timeout -k 10 300 python -u -m pytest tests/test_kd_fold_gpu.py tests/test_misc_ops_gpu.py -k "kd" -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_kd3/tests.log 2>&1 || { tail -30 gpurun_out/r6_kd3/tests.log; exit 1; }
tail -1 gpurun_out/r6_kd3/tests.log
for f in 1 0 1; do
RTSEG_KD_FOLD=$f timeout -k 10 500 python -u bench.py --kd --batch 16 --steps 10 --warmup 4 --no-infer > gpurun_out/r6_kd3/bench_kd_f$f.json 2> gpurun_out/r6_kd3/bench_kd_f$f.err || { tail -20 gpurun_out/r6_kd3/bench_kd_f$f.err; exit 1; }
echo "fold=$f $(tail -1 gpurun_out/r6_kd3/bench_kd_f$f.json | cut -c1-110)"
done
for d in 0 8 16; do RTSEG_HREG_DBG=$d timeout -k 10 200 python -u tools/bench_hreg.py > gpurun_out/r6_kd3/hreg_dbg$d.txt 2>&1 || exit 1; done
