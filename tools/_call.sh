set -o pipefail
mkdir -p gpurun_out/r6_kd
timeout -k 10 500 python -u bench.py --kd --batch 16 --steps 10 --warmup 4 --no-infer > gpurun_out/r6_kd/bench_kd_b16.json 2> gpurun_out/r6_kd/bench_kd.err || { tail -20 gpurun_out/r6_kd/bench_kd.err; exit 1; }
tail -1 gpurun_out/r6_kd/bench_kd_b16.json | cut -c1-200
PROF_SKIP=4 PROF_PER_STEP=2 timeout -k 10 600 bash tools/profile_bench.sh gpurun_out/r6_kd/prof --kd --batch 16 --steps 6 --warmup 4 > gpurun_out/r6_kd/prof.log 2>&1 || { tail -20 gpurun_out/r6_kd/prof.log; exit 1; }
rm -f gpurun_out/r6_kd/prof/trace.csv.gz
head -50 gpurun_out/r6_kd/prof/steady.txt | cut -c1-170
