set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/r6_tune2; mkdir -p $D
cp miopen_db/rtseg_conv_decisions.json $D/db.json
RTSEG_TUNE_DB_OUT=$D/db.json timeout -k 10 600 python -u bench.py --model bisenetv2 --batch 16 --steps 10 --warmup 3 --no-infer > $D/bisenetv2.json 2> $D/bisenetv2.err || { tail -20 $D/bisenetv2.err; exit 1; }
cut -c1-160 $D/bisenetv2.json
RTSEG_TUNE_DB_OUT=$D/db.json timeout -k 10 600 python -u bench.py --model stdc --arch stdc2 --detail-head --batch 16 --steps 10 --warmup 3 --no-infer > $D/stdc2.json 2> $D/stdc2.err || { tail -20 $D/stdc2.err; exit 1; }
cut -c1-160 $D/stdc2.json
RTSEG_TUNE_DB_OUT=$D/db.json timeout -k 10 600 python -u bench.py --kd --batch 16 --steps 10 --warmup 3 --no-infer > $D/kd.json 2> $D/kd.err || { tail -20 $D/kd.err; exit 1; }
cut -c1-160 $D/kd.json
