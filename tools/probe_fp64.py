"""Whole-model gradient accuracy: GPU HIP path and GPU torch path vs a CPU fp64 run."""
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
    return ((a.double().cpu() - b.double().cpu()).norm() / (b.double().cpu().norm() + 1e-30)).item()


def run(m, x, labels, disable=False):
    os.environ["RTSEG_DISABLE_HIP"] = "1" if disable else "0"
    torch.manual_seed(123)
    with ops.defer_final_upsample():
        out = m(x, is_training=True)
    out = out[0] if isinstance(out, (tuple, list)) else out
    loss = SegCELoss(ops.MODE_MEAN)(out, labels)
    loss.backward()
    os.environ["RTSEG_DISABLE_HIP"] = "0"
    return loss.item(), {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}


for key in sys.argv[1:]:
    c = BaseConfig()
    c.model, c.num_class, c.use_aux, c.use_detail_head = key, 19, False, False
    torch.manual_seed(0)
    base = get_model(c).train()
    x = torch.randn(2, 3, 128, 256)
    labels = torch.randint(0, 19, (2, 128, 256))
    l64, g64 = run(copy.deepcopy(base).double(), x.double(), labels)
    gb = copy.deepcopy(base).cuda().to(memory_format=torch.channels_last)
    xg = x.cuda().contiguous(memory_format=torch.channels_last)
    lh, gh = run(copy.deepcopy(gb), xg, labels.cuda())
    lt, gt = run(copy.deepcopy(gb), xg, labels.cuda(), True)
    cat = lambda g: torch.cat([g[n].flatten().double().cpu() for n in g64])  # noqa: E731
    print(f"{key:12s} loss fp64 {l64:.6f} hip {lh:.6f} torch {lt:.6f} | grads hip {rel(cat(gh), cat(g64)):.2e} "
          f"torch {rel(cat(gt), cat(g64)):.2e}", flush=True)
    worst = sorted(((rel(gh[n], g64[n]), rel(gt[n], g64[n]), n) for n in g64), reverse=True)[:5]
    for eh, et, n in worst:
        print(f"      hip {eh:.2e} torch {et:.2e} {n} |g|={g64[n].norm():.2e}", flush=True)
