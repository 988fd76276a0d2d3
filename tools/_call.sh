set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
D=gpurun_out/r6_stemeval; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_conv_stem_gpu.py -v --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { grep -E "FAILED|^E  " $D/tests.log | head -30; tail -3 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for i in 1 2; do
timeout -k 10 180 python3 tools/profile_infer.py --iters 300 > $D/infer_$i.txt 2>&1 || { tail -5 $D/infer_$i.txt; exit 1; }
echo "$(tail -1 $D/infer_$i.txt)"
done
timeout -k 10 180 python3 - > $D/decisions.txt 2>&1 <<'PY'
import sys, os
sys.path.insert(0, os.getcwd())
import torch
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
from realtime_semantic_segmentation_pytorch_amd.models import get_model
from realtime_semantic_segmentation_pytorch_amd.utils.inference import InferenceEngine
from realtime_semantic_segmentation_pytorch_amd.ops import conv as cm
c = BaseConfig(); c.model, c.arch_type, c.num_class, c.use_aux = "ddrnet", "DDRNet-23", 19, True
m = get_model(c).cuda()
eng = InferenceEngine(m, (1, 3, 1024, 2048), dtype=torch.bfloat16, warmup=3)
for k, v in sorted(cm._DECISIONS.items(), key=lambda kv: repr(kv[0])):
    print(k, v[1], v[2])
PY
grep -c eval $D/decisions.txt; grep "wres\|igemm_k\|miopen" $D/decisions.txt | head -30
