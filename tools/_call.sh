set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/r6_haloeval; mkdir -p $D
cp miopen_db/rtseg_conv_decisions.json $D/db.json
for i in 1 2; do for v in auto 0; do
if [ $v = auto ]; then OUTV="RTSEG_TUNE_DB_OUT=$D/db.json"; else OUTV=""; fi
env $OUTV RTSEG_CONV_HALO=$v timeout -k 10 180 python3 tools/profile_infer.py --iters 300 > $D/infer_${v}_$i.txt 2>&1 || { tail -5 $D/infer_${v}_$i.txt; exit 1; }
echo "halo=$v $(tail -1 $D/infer_${v}_$i.txt)"
done; done
