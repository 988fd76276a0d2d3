set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/r6_tune; mkdir -p $D
RTSEG_TUNE_DB_OUT=$D/db.json timeout -k 10 600 python -u bench.py > $D/bench1.json 2> $D/bench1.err || { tail -20 $D/bench1.err; exit 1; }
cut -c1-200 $D/bench1.json
RTSEG_TUNE_DB=$D/db.json timeout -k 10 600 python -u bench.py > $D/bench2.json 2> $D/bench2.err || { tail -20 $D/bench2.err; exit 1; }
cat $D/bench2.json
