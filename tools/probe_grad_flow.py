"""Localise a backward discrepancy: HIP path vs torch path, per leaf module.

Records grad_output / grad_input of every leaf module (full backward hooks) in
both paths and prints, in backward order, modules whose grad_input deviates
while their grad_output still agrees -- the op that introduces the error.
"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import copy

import torch

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
from realtime_semantic_segmentation_pytorch_amd.core.loss import SegCELoss
from realtime_semantic_segmentation_pytorch_amd.models import get_model


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def run(m, x, labels, disable):
    os.environ["RTSEG_DISABLE_HIP"] = "1" if disable else "0"
    rec = []
    hooks = []
    for name, mod in m.named_modules():
        if len(list(mod.children())) == 0:
            def hook(mod, gin, gout, name=name):
                gi = gin[0].detach().clone() if gin and gin[0] is not None else None
                go = gout[0].detach().clone() if gout and gout[0] is not None else None
                rec.append((name, type(mod).__name__, go, gi))
            hooks.append(mod.register_full_backward_hook(hook))
    torch.manual_seed(123)
    with ops.defer_final_upsample():
        out = m(x, is_training=True)
    out = out[0] if isinstance(out, (tuple, list)) else out
    SegCELoss(ops.MODE_MEAN)(out, labels).backward()
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    os.environ["RTSEG_DISABLE_HIP"] = "0"
    return rec


key = sys.argv[1]
c = BaseConfig()
c.model, c.num_class, c.use_aux, c.use_detail_head = key, 19, False, False
torch.manual_seed(0)
base = get_model(c).cuda().to(memory_format=torch.channels_last).train()
x = torch.randn(2, 3, 128, 256, device="cuda").contiguous(memory_format=torch.channels_last)
labels = torch.randint(0, 19, (2, 128, 256), device="cuda")
rh = run(copy.deepcopy(base), x, labels, False)
rt = run(copy.deepcopy(base), x, labels, True)
print(len(rh), len(rt))
for (n, t, goh, gih), (_, _, got, git) in zip(rh, rt):
    eo = rel(goh, got) if goh is not None and got is not None else float("nan")
    ei = rel(gih, git) if gih is not None and git is not None else float("nan")
    flag = " <<<" if ei > 1e-3 and not eo > 1e-4 else ""
    info = f" go {tuple(goh.shape)} {goh.stride()} {goh.dtype}" if goh is not None else ""
    info += f" gi {gih.stride()}" if gih is not None else ""
    print(f"{n:45s} {t:18s} gout {eo:.2e} gin {ei:.2e}{flag}{info}", flush=True)
