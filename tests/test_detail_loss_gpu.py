"""Fused STDC detail loss (csrc/kernels/detail_loss.hip) vs the fp32 PyTorch formulation of the
reference (Laplacian target, 1x1 fuse, threshold, x8 bilinear resize, Dice on raw logits + BCE)."""
import pytest
import torch
import torch.nn as nn

from realtime_semantic_segmentation_pytorch_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _lib():
    assert ops.load(), "HIP extension must load on the GPU box"


def _labels(n, h, w, dtype, seed=0):
    torch.manual_seed(seed)
    # blocky class map with ignore (255) regions: edges at several scales
    lab = torch.randint(0, 19, (n, h // 16 + 1, w // 16 + 1), device=DEV)
    lab = lab.repeat_interleave(16, 1).repeat_interleave(16, 2)[:, :h, :w].contiguous()
    lab[:, : h // 5, : w // 7] = 255
    return lab.to(dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ldtype", [torch.uint8, torch.int64])
@pytest.mark.parametrize("n,h,w", [(2, 128, 256), (1, 100, 76), (3, 64, 200)])
def test_detail_loss_matches_reference(dtype, ldtype, n, h, w):
    conv = nn.Conv2d(3, 1, 1, bias=False).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(torch.tensor([0.5, 0.3, 0.2], device=DEV).view(1, 3, 1, 1))
    labels = _labels(n, h, w, ldtype)
    torch.manual_seed(1)
    d = (torch.randn(n, 1, (h + 7) // 8, (w + 7) // 8, device=DEV) * 2).to(dtype).requires_grad_(True)
    loss = ops.detail_loss(d, labels, conv, 0.1, 1.0, 1.0)
    dr = d.detach().float().requires_grad_(True)
    ref = ops.detail_loss_reference(dr, labels.long(), conv, 0.1, 1.0, 1.0)
    torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-5)
    loss.backward(torch.tensor(0.5, device=DEV))
    ref.backward(torch.tensor(0.5, device=DEV))
    scale = dr.grad.abs().max().item()
    tol = 1e-4 if dtype == torch.float32 else 1e-2
    torch.testing.assert_close(d.grad.float(), dr.grad, atol=tol * scale, rtol=tol)


def test_detail_target_is_exact():
    conv = nn.Conv2d(3, 1, 1, bias=True).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(torch.tensor([1.0, -0.5, 0.25], device=DEV).view(1, 3, 1, 1))
        conv.bias.fill_(0.05)
    labels = _labels(2, 96, 160, torch.int64, seed=4)
    y = ops.detail_target_reference(labels, conv, 0.1)
    # zero logits: BCE = log 2 everywhere, Dice depends only on sum(gt) -> checks the target count
    d = torch.zeros(2, 1, 12, 20, device=DEV)
    loss = ops.detail_loss(d, labels, conv, 0.1, 1.0, 0.0)
    want = (1 - 1 / (y.flatten(1).sum(1) + 1)).mean()
    torch.testing.assert_close(loss, want, rtol=1e-6, atol=1e-6)
