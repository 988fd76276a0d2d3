set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/r6_infer4; mkdir -p $D
timeout -k 10 180 python3 tools/profile_infer.py --iters 200 > $D/wall.txt 2>&1 || { tail -5 $D/wall.txt; exit 1; }
wall=$(grep -o "[0-9.]* ms/img" $D/wall.txt | tail -1 | cut -d' ' -f1)
RAW=/tmp/rtseg_lat_ddr; rm -rf $RAW
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $RAW -o run -- python3 tools/profile_infer.py --iters 200 > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
TRACE=$(find $RAW -name "*kernel_trace.csv" | head -1)
python3 tools/latency_report.py "$TRACE" --iters 200 --wall-ms "$wall" --top 40 > $D/report.txt || exit 1
gzip -c $TRACE > $D/trace.csv.gz
cat $D/wall.txt | tail -1; head -8 $D/report.txt
