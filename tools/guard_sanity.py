"""Sanity of the guard-page allocator itself (RTSEG_GUARD=tail): basic torch ops on guard memory
vs the same ops on the CPU.  python tools/guard_sanity.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd.utils import guard  # noqa: E402

guard.install(os.environ.get("RTSEG_GUARD", "tail"))
torch.backends.cudnn.enabled = os.environ.get("GUARD_CUDNN", "0") == "1"


def rel(a, b):
    return ((a.double().cpu() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


g = torch.Generator().manual_seed(0)
xc = torch.randn(4, 8, 32, 48, generator=g)
x = xc.cuda()
print("h2d->d2h", rel(x, xc), flush=True)
print("add", rel(x + 1, xc + 1), flush=True)
print("sum", rel(x.sum(), xc.sum()), flush=True)
a, b = torch.randn(64, 96, generator=g), torch.randn(96, 80, generator=g)
print("mm", rel(a.cuda() @ b.cuda(), a @ b), flush=True)
w = torch.randn(16, 8, 3, 3, generator=g)
print("conv", rel(torch.nn.functional.conv2d(x, w.cuda(), padding=1), torch.nn.functional.conv2d(xc, w, padding=1)),
      flush=True)
r = torch.randn(3, 1000, generator=g)
print("randn-gpu finite", bool(torch.isfinite(torch.randn(1000, device="cuda")).all()), flush=True)
y = torch.empty(1000, device="cuda")
y.copy_(r[0].cuda())
print("copy", rel(y, r[0]), flush=True)
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402

xi = xc.contiguous(memory_format=torch.channels_last)
print("rtseg interp", rel(ops.interpolate(xi.cuda(), (64, 96), True), torch.nn.functional.interpolate(
    xc, (64, 96), mode="bilinear", align_corners=True)), flush=True)
print("stats", guard.stats(), flush=True)
