"""Transposed conv on the MFMA kernels (ops/deconv.py) and the gather-form indexed max pool /
max unpool (ops/pool.py, pool.hip) vs fp32 PyTorch, forward and backward.
Reference sites: models/modules.py:89-108 (DeConvBNAct), enet.py:119-184, segnet.py:45-80."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _lib():
    assert ops.load(), "HIP extension must load on the GPU box"


def _close(got, ref, tol):
    torch.testing.assert_close(got.float(), ref.float(), atol=tol * ref.float().abs().max().item() + 1e-6, rtol=tol)


# (n, cin_t, cout_t, h, w, k, stride, pad, out_pad): DeConvBNAct x2 / x4, ENet's upsampler, a
# backward that falls back (cout_t % 64 != 0)
DECONV = [
    (2, 64, 64, 17, 23, 3, 2, 1, 1),
    (2, 128, 64, 9, 12, 7, 4, 3, 3),
    (1, 128, 128, 8, 10, 3, 2, 1, 1),
    (2, 64, 16, 11, 7, 3, 2, 1, 1),
]


@pytest.mark.parametrize("geom", DECONV)
def test_transposed_conv_matches_torch(geom):
    n, ci, co, h, w, k, s, p, op = geom
    g = torch.Generator().manual_seed(0)
    m = ops.TransposedConv2d(ci, co, k, s, p, op).to(DEV)
    with torch.no_grad():
        m.weight.copy_(torch.randn(m.weight.shape, generator=g) / (ci * k * k / s / s) ** 0.5)
        m.bias.copy_(torch.randn(co, generator=g) * 0.1)
    x = torch.randn(n, ci, h, w, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    x = x.to(torch.bfloat16).requires_grad_(True)
    assert ops.deconv_ok(x, m)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    ref_x = x.detach().float().requires_grad_(True)
    wref = m.weight.detach().clone().requires_grad_(True)
    bref = m.bias.detach().clone().requires_grad_(True)
    ref = F.conv_transpose2d(ref_x, wref, bref, s, p, op)
    assert y.shape == ref.shape
    _close(y, ref, 2e-2)
    gy = torch.randn(ref.shape, generator=g).to(DEV)
    y.float().backward(gy)
    ref.backward(gy)
    _close(x.grad, ref_x.grad, 3e-2)
    _close(m.weight.grad, wref.grad, 2e-2)
    _close(m.bias.grad, bref.grad, 2e-2)  # dy arrives in bf16


def test_deconvbnact_module_routes_through_hip():
    from realtime_semantic_segmentation_pytorch_amd.models.modules import DeConvBNAct

    blk = ops.convert_transposed_convs(ops.convert_batchnorm(DeConvBNAct(128, 64))).to(DEV).train()
    assert isinstance(blk.up_conv[0], ops.TransposedConv2d)
    x = torch.randn(2, 128, 16, 24, device=DEV).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = blk(x)
    assert y.shape == (2, 64, 32, 48) and torch.isfinite(y.float()).all()


@pytest.mark.parametrize("channels_last", [True, False])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("hw", [(16, 24), (15, 21)])
def test_max_pool_indices_and_unpool(channels_last, dtype, hw):
    h, w = hw
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 24, h, w, generator=g).to(DEV, dtype)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    pool = ops.MaxPool2d(2, 2, return_indices=True)
    unpool = ops.MaxUnpool2d(2, 2)
    y, idx = pool(x)
    xr = x.detach().float().requires_grad_(True)
    yr, idxr = F.max_pool2d(xr, 2, 2, return_indices=True)
    assert idx.dtype == torch.int64 and torch.equal(idx.cpu(), idxr.cpu())
    _close(y, yr, 0)
    z = torch.randn(y.shape, generator=g).to(DEV, dtype).requires_grad_(True)
    u = unpool(z, idx, output_size=x.shape)
    zr = z.detach().float().requires_grad_(True)
    ur = F.max_unpool2d(zr, idxr, 2, 2, output_size=x.shape[2:])
    assert u.shape == ur.shape
    _close(u, ur, 0)
    gu = torch.randn(u.shape, generator=g).to(DEV, dtype)
    (u.float() * gu.float()).sum().backward()
    (ur * gu.float()).sum().backward()
    _close(z.grad, zr.grad, 0)
    gy = torch.randn(y.shape, generator=g).to(DEV, dtype)
    (y.float() * gy.float()).sum().backward()
    (yr * gy.float()).sum().backward()
    _close(x.grad, xr.grad, 0)


@pytest.mark.parametrize("model", ["enet", "segnet"])
def test_enet_segnet_indexed_pool_train_step(model):
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.models import get_model

    c = BaseConfig()
    c.model, c.num_class = model, 19
    net = get_model(c).to(DEV).to(memory_format=torch.channels_last).train()
    assert any(isinstance(m, ops.MaxUnpool2d) for m in net.modules())
    x = torch.randn(2, 3, 128, 256, device=DEV).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = net(x)
    out.float().mean().backward()
    assert torch.isfinite(out.float()).all()
    assert all(torch.isfinite(p.grad).all() for p in net.parameters() if p.grad is not None)


@pytest.mark.parametrize("channels_last", [True, False])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_global_max_pool(channels_last, dtype):
    g = torch.Generator().manual_seed(2)
    x = torch.randn(3, 150, 9, 13, generator=g).to(DEV, dtype)
    x[0, 3, 2, 2] = x[0, 3, 5, 7] = 50.0  # tie: the first pixel wins
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = ops.AdaptiveMaxPool2d(1)(x)
    xr = x.detach().float().requires_grad_(True)
    yr = F.adaptive_max_pool2d(xr, 1)
    _close(y, yr, 0)
    gy = torch.randn(y.shape, generator=g).to(DEV, dtype)
    (y.float() * gy.float()).sum().backward()
    (yr * gy.float()).sum().backward()
    _close(x.grad, xr.grad, 0)
