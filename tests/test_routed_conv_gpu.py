"""Plain dense convs a model calls directly (``ops.RoutedConv2d``, ``ops.convert_routed_convs``):
bf16 training forward + backward through the routed conv node vs an fp32 PyTorch conv of the same
bf16-rounded operands, and bf16 inference through the cached bf16 weight.

Reference sites: ERFNet's non-bottleneck-1D tail conv (reference models/erfnet.py), STDC's
``conv4`` / ``conv5`` (reference models/stdc.py:13-101) -- ``nn.Conv2d`` modules outside any
ConvBNAct."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (n, cin, h, w, cout, kernel, stride, padding, dilation)
GEOMS = [
    (2, 64, 24, 40, 64, (1, 3), 1, (0, 2), (1, 2)),    # ERFNet factorised, dilated
    (2, 128, 16, 32, 128, (3, 1), 1, (4, 0), (4, 1)),
    (2, 512, 8, 16, 256, 1, 1, 0, 1),                  # STDC conv4
    (1, 64, 33, 17, 128, 3, 2, 1, 1),
    (2, 96, 20, 20, 64, 3, 1, 1, 1),                   # Cin % 64 != 0: the 16x16x32 family
]


@pytest.fixture(autouse=True)
def _lib():
    assert ops.load(), "HIP extension must load on the GPU box"


def _close(got, ref, tol):
    torch.testing.assert_close(got.float(), ref, atol=tol * ref.abs().max().item() + 1e-6, rtol=tol)


@pytest.mark.parametrize("geom", GEOMS)
def test_routed_conv_training_matches_fp32(geom):
    n, cin, h, w, cout, k, s, p, d = geom
    torch.manual_seed(0)
    conv = nn.Conv2d(cin, cout, k, s, p, d, bias=False)
    ops.convert_routed_convs(nn.Sequential(conv))
    assert type(conv) is ops.RoutedConv2d
    conv = conv.to(DEV).to(memory_format=torch.channels_last).train()
    x = torch.randn(n, cin, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = conv(x)
    assert y.grad_fn is not None and "ConvFn" in type(y.grad_fn).__name__, type(y.grad_fn).__name__
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_(True)
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    ref = F.conv2d(xr, wr, None, s, p, d)
    ref.backward(g.float())
    _close(y, ref.detach(), 2e-2)
    _close(x.grad, xr.grad, 3e-2)
    _close(conv.weight.grad, wr.grad, 3e-2)
    assert conv.weight.grad.stride() == conv.weight.stride()


@pytest.mark.parametrize("geom", GEOMS[:3])
def test_routed_conv_inference_uses_cached_bf16_weight(geom):
    n, cin, h, w, cout, k, s, p, d = geom
    conv = nn.Conv2d(cin, cout, k, s, p, d, bias=False)
    ops.convert_routed_convs(nn.Sequential(conv))
    conv = conv.to(DEV).to(memory_format=torch.channels_last).eval()
    x = torch.randn(n, cin, h, w, device=DEV).contiguous(memory_format=torch.channels_last)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y = conv(x)
        y2 = conv(x)
    assert getattr(conv, "_rtseg_w16", None) is not None
    ref = F.conv2d(x.to(torch.bfloat16).float(), conv.weight.to(torch.bfloat16).float(), None, s, p, d)
    _close(y, ref, 2e-2)
    torch.testing.assert_close(y, y2)


@pytest.mark.parametrize("k,dil", [(1, 1), (3, 1), ((3, 1), (4, 1))])
def test_biased_conv_bias_add_matches_conv2d(k, dil):
    """Biased dense convs (PrunedConv2d after ops.convert_pruned_convs): bias-free conv + bias_add,
    whose bias gradient is the HIP channel-sum pass, == F.conv2d with the bias (fp32 and bf16)."""
    from realtime_semantic_segmentation_pytorch_amd.ops.dilated import PrunedConv2d, convert_pruned_convs

    torch.manual_seed(0)
    kk = k if isinstance(k, tuple) else (k, k)
    pad = tuple((a - 1) // 2 * d for a, d in zip(kk, dil if isinstance(dil, tuple) else (dil, dil)))
    conv = torch.nn.Conv2d(32, 48, kk, padding=pad, dilation=dil, bias=True).cuda()
    ref = copy.deepcopy(conv)
    convert_pruned_convs(conv)
    assert type(conv) is PrunedConv2d
    for dtype in (torch.float32, torch.bfloat16):
        x = torch.randn(2, 32, 24, 40, device="cuda").contiguous(memory_format=torch.channels_last)
        outs = []
        for m in (conv, ref):
            m.zero_grad()
            xx = x.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
                y = m(xx)
            g = torch.randn(y.shape, device="cuda", generator=torch.Generator("cuda").manual_seed(1))
            (y.float() * g).sum().backward()
            outs.append((y.float(), xx.grad.float(), m.weight.grad.float(), m.bias.grad.float()))
        tol = 1e-4 if dtype == torch.float32 else 2e-2
        for a, b in zip(*outs):
            assert float((a - b).norm() / (b.norm() + 1e-12)) < tol


# (n, c, h, w, groups, stride, dilation, split): RegSeg D-block grouped 3x3s (group width 16),
# ``split``: the input is the second channel half of a channels-last tensor (conv_right)
GROUPED = [(2, 128, 16, 24, 8, 1, 2, True), (2, 64, 17, 20, 4, 2, 1, False), (1, 48, 12, 16, 3, 2, 1, False),
           (2, 128, 10, 12, 8, 1, 11, False)]


@pytest.mark.parametrize("geom", GROUPED)
def test_grouped_conv_block_diagonal_route(geom):
    """Training grouped conv through the block-diagonal dense route vs fp32 grouped F.conv2d."""
    n, c, h, w, groups, s, d, split = geom
    torch.manual_seed(0)
    conv = nn.Conv2d(c, c, 3, s, d, d, groups=groups, bias=False).to(DEV).to(memory_format=torch.channels_last)
    src = torch.randn(n, 2 * c if split else c, h, w, device=DEV).to(torch.bfloat16)
    src = src.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    x = src[:, c:] if split else src
    assert ops.conv.grouped_dense_ok(x, conv)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops.conv_forward(x, conv)
    if c % 64 == 0:
        assert "ConvFn" in type(y.grad_fn).__name__, type(y.grad_fn).__name__
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_(True)
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    ref = F.conv2d(xr, wr, None, s, d, d, groups)
    ref.backward(g.float())
    _close(y, ref.detach(), 2e-2)
    gx = src.grad[:, c:] if split else src.grad
    _close(gx, xr.grad, 3e-2)
    _close(conv.weight.grad, wr.grad, 3e-2)


def _ref_grads(x, w, g, fn):
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().to(torch.bfloat16).float().requires_grad_(True)
    ref = fn(xr, wr)
    ref.backward(g.float())
    return ref.detach(), xr.grad, wr.grad


@pytest.mark.parametrize("raw", [False, True])
def test_padded_cout_route(raw):
    """SegNet's 3x3 19-class classifier: Cout % 8 != 0 runs on the weight zero-padded to 64 output
    channels (ops/conv.py padded_ok / _apply) -- through the ConvBNAct statistics path and as a
    plain RoutedConv2d."""
    torch.manual_seed(0)
    conv = nn.Conv2d(64, 19, 3, 1, 1, bias=False)
    if raw:
        ops.convert_routed_convs(nn.Sequential(conv))
    conv = conv.to(DEV).to(memory_format=torch.channels_last).train()
    assert ops.conv.padded_ok(conv)
    x = torch.randn(2, 64, 20, 36, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = conv(x) if raw else ops.conv_bn_stats(x, conv)[0]
    assert y.shape == (2, 19, 20, 36) and y.is_contiguous(memory_format=torch.channels_last)
    g = torch.randn_like(y)
    y.backward(g)
    ref, gx, gw = _ref_grads(x, conv.weight, g, lambda a, b: F.conv2d(a, b, None, 1, 1))
    _close(y, ref, 2e-2)
    _close(x.grad, gx, 3e-2)
    _close(conv.weight.grad, gw, 3e-2)


@pytest.mark.parametrize("geom", [(64, 16, 1, 4, 1), (256, 64, 1, 4, 1), (128, 128, 3, 8, 4)])
def test_grouped_module_routes(geom):
    """Grouped convs called as plain modules: ESPNetv2's EESP 1x1 (groups 4) -> GroupedConv2d,
    RegSeg's dilated D-block conv -> DilatedGroupConv2d; both train on the block-diagonal route."""
    cin, cout, k, groups, dil = geom
    torch.manual_seed(0)
    conv = nn.Conv2d(cin, cout, k, 1, dil * (k // 2), dil, groups=groups, bias=False)
    ops.convert_dilated_group_convs(nn.Sequential(conv))
    ops.convert_routed_convs(nn.Sequential(conv))
    assert type(conv) is (ops.DilatedGroupConv2d if dil > 1 else ops.GroupedConv2d), type(conv)
    conv = conv.to(DEV).to(memory_format=torch.channels_last).train()
    x = torch.randn(2, cin, 24, 40, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = conv(x)
    assert "ConvFn" in type(y.grad_fn).__name__, type(y.grad_fn).__name__
    g = torch.randn_like(y)
    y.backward(g)
    ref, gx, gw = _ref_grads(x, conv.weight, g, lambda a, b: F.conv2d(a, b, None, 1, dil * (k // 2), dil, groups))
    _close(y, ref, 2e-2)
    _close(x.grad, gx, 3e-2)
    _close(conv.weight.grad, gw, 3e-2)
