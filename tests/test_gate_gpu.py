"""Attention gating kernels (gate.hip via ops.gate) vs fp32 PyTorch, forward and backward, for
the three broadcast forms and three modes.  Reference sites: bisenetv1.py:76-114,
regseg.py:109-127, pp_liteseg.py:120-141, bisenetv2.py:140-162."""
import pytest
import torch

from realtime_semantic_segmentation_pytorch_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _lib():
    assert ops.load(), "HIP extension must load on the GPU box"


def _close(got, ref, tol):
    torch.testing.assert_close(got.float(), ref.float(), atol=tol * ref.float().abs().max().item() + 1e-5, rtol=tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("bcast", ["channel", "spatial", "full"])
@pytest.mark.parametrize("mode", ["mul", "residual", "blend"])
@pytest.mark.parametrize("sigmoid", [False, True])
@pytest.mark.parametrize("c", [64, 24])
def test_gate_matches_torch(dtype, bcast, mode, sigmoid, c):
    g = torch.Generator().manual_seed(0)
    n, h, w = 2, 13, 17
    cl = dict(memory_format=torch.channels_last)
    x = torch.randn(n, c, h, w, generator=g).to(DEV, dtype).contiguous(**cl).requires_grad_(True)
    other = torch.randn(n, c, h, w, generator=g).to(DEV, dtype).contiguous(**cl).requires_grad_(True)
    shape = {"channel": (n, c, 1, 1), "spatial": (n, 1, h, w), "full": (n, c, h, w)}[bcast]
    att = torch.randn(shape, generator=g).to(DEV)
    if not sigmoid:
        att = torch.sigmoid(att)
    att = (att.to(dtype).contiguous(**cl) if bcast == "full" else att).requires_grad_(True)
    o = other if mode == "blend" else None
    y = ops.gate(x, att, o, mode, sigmoid)
    assert y.dtype == dtype and y.shape == x.shape
    xr, orr, ar = (t.detach().float().requires_grad_(True) for t in (x, other, att))
    ref = ops.gate_reference(xr, ar, orr if mode == "blend" else None, mode, sigmoid)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    _close(y, ref, tol)
    gy = torch.randn(ref.shape, generator=g).to(DEV)
    (y.float() * gy).sum().backward()
    (ref * gy).sum().backward()
    _close(x.grad, xr.grad, tol)
    _close(att.grad, ar.grad, 1e-4 if dtype == torch.float32 else 3e-2)
    if mode == "blend":
        _close(other.grad, orr.grad, tol)


def test_gate_takes_the_hip_path():
    x = torch.randn(2, 32, 8, 8, device=DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    att = torch.rand(2, 32, 1, 1, device=DEV, requires_grad=True)
    y = ops.gate(x, att)
    assert type(y.grad_fn).__name__ == "_GateFnBackward"
