"""Fused BatchNorm(+residual)+activation HIP kernels vs PyTorch BatchNorm (fp64 / fp32)."""
import copy

import pytest
import torch
import torch.nn as nn

from realtime_semantic_segmentation_pytorch_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(x, bn, act, res):
    y = bn(x)
    if res is not None:
        y = y + res
    if act == "relu":
        y = torch.relu(y)
    elif act == "relu6":
        y = torch.nn.functional.relu6(y)
    return y


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", ["none", "relu", "relu6"])
@pytest.mark.parametrize("with_res", [False, True])
@pytest.mark.parametrize("shape", [(2, 64, 17, 33), (3, 256, 8, 8), (1, 1024, 4, 6), (4, 16, 32, 32),
                                   (2, 12, 9, 10), (2, 19, 16, 16), (2, 3, 5, 7), (2, 250, 1, 1), (3, 131, 4, 4),
                                   (2, 36, 8, 8)])
def test_bn_act_train(dtype, act, with_res, shape):
    assert ops.load()
    torch.manual_seed(0)
    c = shape[1]
    bn = nn.BatchNorm2d(c).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    # fp64 reference: torch's fp32 BN is itself ~1e-4 off at 2 values per channel with var ~ eps
    bn_ref = copy.deepcopy(bn).double()
    x = (torch.randn(shape, device=DEV) * 2 + 0.5).to(dtype).contiguous(memory_format=torch.channels_last)
    res = (torch.randn(shape, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
           if with_res else None)
    x.requires_grad_(True)
    if res is not None:
        res.requires_grad_(True)
    assert ops.bn_fused_ok(x, bn, ops.bn_act_code(act))  # the HIP path, not the fallback
    y = ops.bn_act(x, bn, act, residual=res)
    xr = x.detach().double().requires_grad_(True)
    rr = res.detach().double().requires_grad_(True) if res is not None else None
    yr64 = _ref(xr, bn_ref, act, rr)
    yr = yr64.detach().float()
    if act != "none":  # compare with the kernel's own activation mask (bf16 rounding at 0 / 6)
        lo = y.detach().float() > 0
        yr = torch.where(lo | (yr <= 0), yr, torch.zeros_like(yr)) if act == "relu" else yr
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    torch.testing.assert_close(bn.running_mean, bn_ref.running_mean.float(), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(bn.running_var, bn_ref.running_var.float(), atol=1e-3, rtol=1e-3)
    assert int(bn.num_batches_tracked) == int(bn_ref.num_batches_tracked) == 1
    g = torch.randn(shape, device=DEV)
    y.backward(g.to(dtype).contiguous(memory_format=torch.channels_last))
    yr64.backward(g.double())
    gt = 2e-3 if dtype == torch.float32 else 6e-2
    scale = xr.grad.float().abs().max().item()
    if dtype == torch.float32 or act == "none":
        torch.testing.assert_close(x.grad.float(), xr.grad.float(), atol=gt * scale, rtol=gt)
    else:  # bf16 mask flips near the kinks: compare the bulk
        bad = ((x.grad.float() - xr.grad.float()).abs() > gt * scale + gt * xr.grad.float().abs()).float().mean()
        assert bad < 2e-3
    torch.testing.assert_close(bn.weight.grad, bn_ref.weight.grad.float(),
                               atol=gt * bn_ref.weight.grad.float().abs().max().item(), rtol=gt)
    torch.testing.assert_close(bn.bias.grad, bn_ref.bias.grad.float(),
                               atol=gt * bn_ref.bias.grad.float().abs().max().item(), rtol=gt)
    if res is not None:
        torch.testing.assert_close(res.grad.float(), rr.grad.float(), atol=gt, rtol=gt)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_act_eval(dtype):
    assert ops.load()
    torch.manual_seed(1)
    bn = nn.BatchNorm2d(32).to(DEV)
    with torch.no_grad():
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    bn.eval()
    x = torch.randn(2, 32, 9, 11, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    y = ops.bn_act(x, bn, "relu")
    yr = torch.relu(bn(x.float()))
    tol = 1e-5 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)


def test_convbnact_module_fused_matches_unfused():
    """ConvBNAct / RB forward+backward: fused GPU path == stock modules (fp32)."""
    from realtime_semantic_segmentation_pytorch_amd.models.ddrnet import RB

    assert ops.load()
    torch.manual_seed(2)
    blk = RB(32, 64, 2).to(DEV).to(memory_format=torch.channels_last)
    ref = copy.deepcopy(blk)
    x = torch.randn(2, 32, 24, 40, device=DEV).contiguous(memory_format=torch.channels_last)
    y = blk(x)
    # reference: plain module math
    s = ref.conv_down[1](ref.conv_down[0](x))
    h = ref.conv1[2](ref.conv1[1](ref.conv1[0](x)))
    yr = torch.relu(ref.conv2[1](ref.conv2[0](h)) + s)
    torch.testing.assert_close(y, yr, atol=1e-4, rtol=1e-4)
    y.sum().backward()
    yr.sum().backward()
    for (n, p), (_, q) in zip(blk.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad, atol=2e-3 * q.grad.abs().max().item() + 1e-6,
                                   rtol=2e-3, msg=n)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 256, 1, 1), (4, 19, 16, 16), (2, 48, 32, 32)])
def test_fused_batchnorm_module_matches_torch(dtype, shape):
    """ops.convert_batchnorm routes plain BatchNorm2d modules (e.g. pooled attention
    branches) through the HIP kernels, train and eval."""
    torch.manual_seed(0)
    ref = nn.BatchNorm2d(shape[1]).to(DEV)
    mod = ops.convert_batchnorm(nn.Sequential(copy.deepcopy(ref)))[0]
    ref.double()  # fp64 reference (torch's fp32 BN is ~4e-4 off at 2 values per channel)
    assert isinstance(mod, ops.FusedBatchNorm2d)
    x = torch.randn(shape, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    assert ops.bn_fused_ok(x, mod, 0)
    for train in (True, False):
        ref.train(train), mod.train(train)
        xa = x.clone().requires_grad_(True)
        xb = x.double().clone().requires_grad_(True)
        ya, yb = mod(xa), ref(xb)
        tol = 1e-4 if dtype == torch.float32 else 3e-2
        torch.testing.assert_close(ya.float(), yb.float(), atol=tol, rtol=tol)
        g = torch.randn(shape, device=DEV)
        ya.backward(g.to(dtype).contiguous(memory_format=torch.channels_last))
        yb.backward(g.double())
        torch.testing.assert_close(xa.grad.float(), xb.grad.float(), atol=10 * tol, rtol=10 * tol)
        # parameter gradients (accumulated over the train and eval passes on both sides)
        for pa, pb in ((mod.weight, ref.weight), (mod.bias, ref.bias)):
            torch.testing.assert_close(pa.grad, pb.grad.float(),
                                       atol=10 * tol * max(1.0, pb.grad.abs().max().item()), rtol=10 * tol)
    torch.testing.assert_close(mod.running_mean, ref.running_mean.float(), atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("act", ["relu", "relu6"])
@pytest.mark.parametrize("shape", [(2, 64, 17, 33), (2, 19, 16, 16), (3, 131, 4, 4)])
def test_bn_residual_bitmask_matches_mask_from_y(monkeypatch, act, shape):
    """Residual + activation backward: the 1-bit derivative mask written by the forward
    (MASK_BITS) gives the same gradients as re-reading the saved output (MASK_FROM_Y)."""
    from realtime_semantic_segmentation_pytorch_amd.ops import bn as bn_mod

    assert ops.load()
    grads = []
    for use_bits in (True, False):
        monkeypatch.setattr(bn_mod, "_USE_BITS", use_bits)
        torch.manual_seed(3)
        bn = nn.BatchNorm2d(shape[1]).to(DEV)
        x = (torch.randn(shape, device=DEV) * 3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        res = torch.randn(shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x.requires_grad_(True)
        res.requires_grad_(True)
        y = ops.bn_act(x, bn, act, residual=res)
        y.backward(torch.randn(shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        grads.append((y.detach(), x.grad, res.grad, bn.weight.grad, bn.bias.grad))
    for a, b in zip(*grads):
        if act == "relu":
            torch.testing.assert_close(a, b, atol=0, rtol=0)
        else:  # relu6: the mask is taken from the fp32 pre-activation vs the bf16-rounded output
            assert ((a.float() - b.float()).abs() > 1e-2 * (1 + b.float().abs())).float().mean() < 1e-3


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act,with_res", [("relu", False), ("relu", True), ("none", False)])
@pytest.mark.parametrize("shape", [(2, 19, 61, 67), (2, 19, 128, 256), (3, 5, 33, 31)])
def test_bn_odd_channels_flat_path(dtype, act, with_res, shape):
    """Odd channel counts (the 19-class full-resolution heads) take the flat, phase-stationary
    kernels: several 16-byte chunks per thread, a partial last chunk, all mask modes.  The fp32
    reference runs on the CPU."""
    assert ops.load()
    torch.manual_seed(1)
    c = shape[1]
    bn = nn.BatchNorm2d(c)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    bn_ref = copy.deepcopy(bn)
    bn = bn.to(DEV)
    x0 = torch.randn(shape) * 2 + 0.5
    r0 = torch.randn(shape) if with_res else None
    x = x0.to(DEV, dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    res = r0.to(DEV, dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True) if with_res else None
    assert ops.bn_fused_ok(x, bn, ops.bn_act_code(act))
    y = ops.bn_act(x, bn, act, residual=res)
    xr = x.detach().float().cpu().requires_grad_(True)
    rr = res.detach().float().cpu().requires_grad_(True) if with_res else None
    yr = _ref(xr, bn_ref, act, rr)
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    if act == "relu":  # compare with the kernel's own activation mask (rounding at 0)
        yr_cmp = torch.where((y.detach().float().cpu() > 0) | (yr <= 0), yr, torch.zeros_like(yr))
    else:
        yr_cmp = yr
    torch.testing.assert_close(y.float().cpu(), yr_cmp.detach(), atol=tol, rtol=tol)
    torch.testing.assert_close(bn.running_mean.cpu(), bn_ref.running_mean, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(bn.running_var.cpu(), bn_ref.running_var, atol=1e-3, rtol=1e-3)
    g = torch.randn(shape)
    y.backward(g.to(DEV, dtype).contiguous(memory_format=torch.channels_last))
    yr.backward(g)
    gt = 2e-3 if dtype == torch.float32 else 6e-2
    scale = xr.grad.abs().max().item()
    bad = ((x.grad.float().cpu() - xr.grad).abs() > gt * scale + gt * xr.grad.abs()).float().mean()
    assert bad < (1e-5 if dtype == torch.float32 else 2e-3)
    torch.testing.assert_close(bn.weight.grad.cpu(), bn_ref.weight.grad,
                               atol=gt * bn_ref.weight.grad.abs().max().item(), rtol=gt)
    torch.testing.assert_close(bn.bias.grad.cpu(), bn_ref.bias.grad,
                               atol=gt * bn_ref.bias.grad.abs().max().item(), rtol=gt)
    if with_res:
        bad_r = ((res.grad.float().cpu() - rr.grad).abs() > gt * rr.grad.abs().max().item()).float().mean()
        assert bad_r < 2e-3


@pytest.mark.parametrize("shape", [(2, 256, 1, 1), (2, 128, 2, 4), (2, 19, 1, 1), (4, 64, 32, 32), (2, 35, 16, 16)])
def test_bn_stats_large_mean_vs_fp64(shape):
    """|mean| >> std (pooled ReLU features: DDRNet's DAPPM global branch, BiSeNetV2's context
    block -- 2 values per channel at batch 2): the shifted one-pass moments keep the batch
    variance, the normalised output and the input gradient at fp32 accuracy against fp64.  With
    plain sum / sum-of-squares partials the variance error was mean^2 / var x 1e-7 (here ~1e-1)."""
    assert ops.load()
    torch.manual_seed(0)
    c = shape[1]
    x64 = (50.0 + 0.05 * torch.randn(shape, dtype=torch.float64)).float().double().to(DEV)  # fp32-exact
    dy = torch.randn(shape, dtype=torch.float64, device=DEV)
    bn = nn.BatchNorm2d(c).to(DEV)
    ref = copy.deepcopy(bn).double()
    xr = x64.clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(dy)
    xh = x64.float().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    yh = ops.bn_act(xh, bn, "none")
    yh.backward(dy.float().contiguous(memory_format=torch.channels_last))
    rel = lambda a, b: ((a.double() - b).norm() / b.norm()).item()  # noqa: E731
    # what remains is fp32 rounding of the folded apply (x * scale + shift with x * scale ~ 1.4e3
    # for an output ~ 1: one fp32 ulp there is 1.2e-4) and of the fp32 mean in the backward's
    # x - mean (50 * 6e-8 / 0.05)
    assert rel(bn.running_var, ref.running_var.double()) < 2e-4
    assert rel(yh.detach(), yr.detach()) < 5e-4
    assert rel(xh.grad, xr.grad) < 5e-4
