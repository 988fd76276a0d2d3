"""Is bf16 inference of a trained DDRNet-23 EMA model deterministic, and do its eval caches match a
fresh copy?  (tests/test_fused_optim_gpu.py::test_ema_validation_sees_new_weights_after_training)"""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_fused_optim_gpu as T  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.datasets import DeviceBatches  # noqa: E402

tr = T._trainer(__import__("pathlib").Path("/tmp/probe_ema"), total_epoch=4)
data = DeviceBatches(2, (128, 256), 19, 255, device=tr.device, pool=1, channels_last=True, seed=2)
imgs, masks = data.next()
x = imgs[:1]


def infer(model):
    model.eval()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        return ops.materialize(model(x)).float()


for _ in range(5):
    tr.train_step(imgs, masks)
a = infer(tr.ema_model.ema)
b = infer(tr.ema_model.ema)
f1 = infer(copy.deepcopy(tr.ema_model.ema))
f2 = infer(copy.deepcopy(tr.ema_model.ema))
for name, u, v in (("cached twice", a, b), ("fresh twice", f1, f2), ("cached vs fresh", a, f1)):
    print(f"{name}: mismatched {int((u != v).sum())} max {float((u - v).abs().max()):.3g}", flush=True)
