"""GPU diagnostic: HIP path vs PyTorch path (RTSEG_DISABLE_HIP=1) per zoo model.

Prints, per model, the relative error of output / loss / all-gradients, the
same numbers for torch-path vs torch-path (run-to-run noise of MIOpen), and
the worst parameters.  Usage: python tools/zoo_parity_report.py [model ...]
"""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.core.loss import SegCELoss  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.models import MODEL_HUB, get_model  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.ops.interp import DeferredLogits  # noqa: E402


def run(m, x, labels, disable):
    os.environ["RTSEG_DISABLE_HIP"] = "1" if disable else "0"
    torch.manual_seed(123)
    with ops.defer_final_upsample():
        out = m(x, is_training=True)
    out = out[0] if isinstance(out, (tuple, list)) else out
    loss = SegCELoss(ops.MODE_MEAN)(out, labels)
    loss.backward()
    full = out.materialize() if isinstance(out, DeferredLogits) else out
    os.environ["RTSEG_DISABLE_HIP"] = "0"
    return full.detach().float(), loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters()
                                                if p.grad is not None}


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    keys = sys.argv[1:] or sorted(MODEL_HUB)
    for key in keys:
        c = BaseConfig()
        c.model, c.num_class, c.use_aux, c.use_detail_head = key, 19, False, False
        torch.manual_seed(0)
        base = get_model(c).cuda().to(memory_format=torch.channels_last).train()
        x = torch.randn(2, 3, 128, 256, device="cuda").contiguous(memory_format=torch.channels_last)
        labels = torch.randint(0, 19, (2, 128, 256), device="cuda")
        yh, lh, gh = run(copy.deepcopy(base), x, labels, False)
        yt, lt, gt = run(copy.deepcopy(base), x, labels, True)
        yt2, lt2, gt2 = run(copy.deepcopy(base), x, labels, True)
        cat = lambda g: torch.cat([v.flatten() for v in g.values()])  # noqa: E731
        gmax = max(v.norm().item() for v in gt.values())
        worst = sorted(((rel(gh[n], gt[n]), n) for n in gt if gt[n].norm() > 1e-3 * gmax), reverse=True)[:4]
        print(f"{key:12s} out {rel(yh, yt):.2e} loss {abs(lh - lt) / abs(lt):.2e} grads {rel(cat(gh), cat(gt)):.2e}"
              f" | noise out {rel(yt2, yt):.2e} grads {rel(cat(gt2), cat(gt)):.2e}", flush=True)
        for e, n in worst:
            print(f"      {e:.2e} {n} |g|={gt[n].norm():.2e} noise {rel(gt2[n], gt[n]):.2e}", flush=True)
        if os.environ.get("ZOO_VERBOSE"):
            for n in gt:  # forward order: the deviation starts downstream of the last clean layer
                print(f"        {rel(gh[n], gt[n]):.2e} (noise {rel(gt2[n], gt[n]):.2e}) {n}", flush=True)


if __name__ == "__main__":
    main()
