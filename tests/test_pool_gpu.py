"""Pooling HIP kernels (csrc/kernels/pool.hip) vs PyTorch fp32 references: avg / max with
fixed windows, adaptive average (incl. the global 1x1 reduction), forward and backward,
channels-last and NCHW, fp32 and bf16."""
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


def _x(shape, dtype, cl, seed=0):
    torch.manual_seed(seed)
    x = torch.randn(shape, device=DEV).to(dtype)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    return x.requires_grad_(True)


def _check(fn, ref, x, dtype):
    y = fn(x)
    # reference in NCHW: ROCm PyTorch's channels-last avg_pool2d backward mis-places the
    # gradient of padded windows (e.g. 6x6, k3 s2 p1 -> row weights 1,1,2,1,2,1 instead
    # of 1,2,1,2,1,1; the CPU and NCHW paths agree with this kernel)
    xr = x.detach().float().contiguous().requires_grad_(True)
    yr = ref(xr)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr).to(dtype).float()  # same rounded upstream gradient for both
    cl = x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous()
    y.backward(g.to(dtype).contiguous(memory_format=torch.channels_last if cl else torch.contiguous_format))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=tol * 2, rtol=tol * 2)
    if cl:
        assert y.is_contiguous(memory_format=torch.channels_last)
        assert x.grad.is_contiguous(memory_format=torch.channels_last)


GEOMS = [((3, 3), 2, 1, True), ((5, 5), 2, 2, True), ((9, 9), 4, 4, True), ((17, 17), 8, 8, True),
         ((3, 3), 2, 1, False), ((2, 2), 2, 0, True), ((3, 1), (2, 1), (1, 0), True)]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [True, False])
@pytest.mark.parametrize("k,s,p,cip", GEOMS)
@pytest.mark.parametrize("shape", [(2, 64, 33, 47), (1, 12, 20, 18)])
def test_avg_pool(dtype, cl, k, s, p, cip, shape):
    x = _x(shape, dtype, cl)
    _check(lambda t: ops.avg_pool2d(t, k, s, p, cip),
           lambda t: F.avg_pool2d(t, k, s, p, count_include_pad=cip), x, dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [True, False])
@pytest.mark.parametrize("k,s,p", [((3, 3), 2, 1), ((2, 2), 2, 0), ((5, 5), 1, 2)])
@pytest.mark.parametrize("shape", [(2, 64, 33, 47), (1, 3, 17, 9)])
def test_max_pool(dtype, cl, k, s, p, shape):
    x = _x(shape, dtype, cl)
    _check(lambda t: ops.max_pool2d(t, k, s, p), lambda t: F.max_pool2d(t, k, s, p), x, dtype)


def test_max_pool_ties_follow_first_maximum():
    torch.manual_seed(3)
    x = F.relu(torch.randn(2, 16, 24, 24, device=DEV)).round().contiguous(memory_format=torch.channels_last)
    a = x.clone().requires_grad_(True)
    b = x.clone().requires_grad_(True)
    g = torch.randn(2, 16, 12, 12, device=DEV)
    ops.max_pool2d(a, 3, 2, 1).backward(g)
    F.max_pool2d(b, 3, 2, 1).backward(g)
    torch.testing.assert_close(a.grad, b.grad)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [True, False])
@pytest.mark.parametrize("out", [1, 2, 4, 6, (3, 5)])
@pytest.mark.parametrize("shape", [(2, 64, 33, 47), (3, 24, 7, 11)])
def test_adaptive_avg_pool(dtype, cl, out, shape):
    x = _x(shape, dtype, cl)
    _check(lambda t: ops.adaptive_avg_pool2d(t, out), lambda t: F.adaptive_avg_pool2d(t, out), x, dtype)


@pytest.mark.parametrize("shape", [(16, 1024, 32, 64), (1, 128, 256, 512), (4, 19, 9, 9)])
def test_global_pool_large(shape):
    x = _x(shape, torch.bfloat16, True)
    _check(lambda t: ops.adaptive_avg_pool2d(t, 1), lambda t: F.adaptive_avg_pool2d(t, 1), x, torch.bfloat16)


def test_convert_pooling_modules():
    m = nn.Sequential(nn.MaxPool2d(3, 2, 1), nn.AvgPool2d(3, 2, 1), nn.AdaptiveAvgPool2d(2),
                      nn.AvgPool2d(3, 2, 1, ceil_mode=True), nn.MaxPool2d(2, return_indices=False, dilation=2))
    ref = [type(c) for c in m]
    ops.convert_pooling(m)
    assert isinstance(m[0], ops.MaxPool2d) and isinstance(m[1], ops.AvgPool2d)
    assert isinstance(m[2], ops.AdaptiveAvgPool2d)
    assert type(m[3]) is ref[3] and type(m[4]) is ref[4]  # unsupported variants keep PyTorch
    x = torch.randn(2, 8, 64, 64, device=DEV).contiguous(memory_format=torch.channels_last)
    y = m[2](m[1](m[0](x)))
    yr = F.adaptive_avg_pool2d(F.avg_pool2d(F.max_pool2d(x, 3, 2, 1), 3, 2, 1), 2)
    torch.testing.assert_close(y, yr, atol=1e-5, rtol=1e-5)
