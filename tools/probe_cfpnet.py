"""Find the source of non-finite gradients in a zoo model's bf16 channels-last train step
(tests/test_zoo.py::test_zoo_bf16_channels_last_train_step_gpu): per seed, report the first
parameters (in registration order) whose gradient is non-finite, plus forward activations."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.core.loss import SegCELoss  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.models import get_model  # noqa: E402

key = sys.argv[1] if len(sys.argv) > 1 else "cfpnet"
for seed in range(int(sys.argv[2]) if len(sys.argv) > 2 else 6):
    torch.manual_seed(seed)
    c = BaseConfig()
    c.model, c.num_class = key, 19
    m = get_model(c).cuda().to(memory_format=torch.channels_last).train()
    bad_act = []

    def hook(mod, inp, out, name=None):
        if isinstance(out, torch.Tensor) and not torch.isfinite(out).all():
            bad_act.append(name)
    for n, mod in m.named_modules():
        mod.register_forward_hook(lambda mod, i, o, n=n: hook(mod, i, o, n))
    x = torch.randn(2, 3, 128, 256, device="cuda").contiguous(memory_format=torch.channels_last)
    labels = torch.randint(0, 19, (2, 128, 256), device="cuda", dtype=torch.uint8)
    loss_fn = SegCELoss(ops.MODE_OHEM, 0.7)
    with torch.autocast("cuda", dtype=torch.bfloat16), ops.defer_final_upsample():
        out = m(x)
        loss = loss_fn(out, labels)
    loss.backward()
    bad = [n for n, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
    print(f"seed {seed}: loss {float(loss):.4f} bad_act {bad_act[:4]} bad_grads {len(bad)} first {bad[:3]} last {bad[-3:]}",
          flush=True)
