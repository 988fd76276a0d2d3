set -o pipefail
D=gpurun_out/r6_det; mkdir -p $D
for i in 1 2; do
for v in 0 1; do
RTSEG_LOSS_ONE_CLASS=$v timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $D/ab_${v}_$i.json 2> $D/ab.err || { tail -20 $D/ab.err; exit 1; }
echo "one_class=$v $(cut -c1-120 $D/ab_${v}_$i.json)"
done; done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python -u bench.py --steps 4 --warmup 3 > $D/prof.log 2>&1 || { tail $D/prof.log; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} grep -E "seg_ce|cast_out" {}
