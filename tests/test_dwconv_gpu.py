"""Depth-wise conv HIP kernels (fwd / dgrad / wgrad) vs F.conv2d in fp32."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.ops.dwconv import DepthwiseConv2d

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (cin, mult, kernel, stride, dilation, hw)
GEOMS = [
    (32, 1, (3, 3), 1, 1, (17, 23)),
    (32, 1, (3, 3), 2, 1, (32, 48)),
    (16, 6, (3, 3), 2, 1, (20, 30)),    # BiSeNetV2 gather-expansion x6
    (24, 1, (3, 1), 1, 2, (15, 9)),     # asymmetric dilated
    (24, 1, (1, 5), 1, 1, (8, 20)),
    (12, 1, (3, 3), 1, 17, (40, 40)),   # large dilation (FDDWNet / LEDNet)
    (3, 1, (3, 3), 1, 1, (9, 11)),      # odd channel count -> scalar vectors
    (40, 2, (5, 5), 1, 1, (12, 14)),    # 25 taps -> several wgrad tap groups
    (64, 1, (3, 3), 1, 1, (64, 128)),
    (8, 5, (3, 3), 1, 1, (10, 12)),     # multiplier without a compiled fast path
    (8, 3, (3, 3), 2, 1, (13, 17)),
    (128, 6, (3, 3), 1, 1, (16, 32)),   # BiSeNetV2 stage-5 shape class
    # round 6: channel-stationary input-pair kernels (fwd / dgrad), the pair wgrad and the
    # stride-2 2x2-block dgrad -- odd sizes hit its edge rows / columns
    (16, 6, (3, 3), 2, 1, (21, 31)),
    (10, 2, (3, 3), 2, 1, (9, 14)),     # 5 input pairs, multiplier 2
    (12, 4, (3, 3), 1, 2, (11, 13)),    # multiplier 4, dilated
    (6, 3, (3, 3), 1, 1, (7, 9)),       # multiplier 3 (odd output vectors)
    (7, 2, (3, 3), 2, 1, (9, 9)),       # odd input channels: no pair path
]


@pytest.fixture(autouse=True)
def _lib():
    assert ops.load(), "HIP extension must load on the GPU box"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("geom", GEOMS)
def test_dwconv_fwd_bwd(dtype, bias, geom):
    cin, mult, k, s, d, hw = geom
    torch.manual_seed(0)
    pad = tuple((kk - 1) // 2 * d for kk in k)
    conv = nn.Conv2d(cin, cin * mult, k, s, pad, d, groups=cin, bias=bias).to(DEV)
    ref = nn.Conv2d(cin, cin * mult, k, s, pad, d, groups=cin, bias=bias).to(DEV)
    ref.load_state_dict(conv.state_dict())
    conv.__class__ = DepthwiseConv2d
    x = torch.randn(2, cin, *hw, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = conv(x)
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().requires_grad_(True)
    yr = ref(xr)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(y.float(), yr, atol=tol * max(1.0, yr.abs().max().item()), rtol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    gt = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=gt * max(1.0, xr.grad.abs().max().item()), rtol=gt)
    torch.testing.assert_close(conv.weight.grad, ref.weight.grad,
                               atol=gt * max(1.0, ref.weight.grad.abs().max().item()), rtol=gt)
    if bias:
        torch.testing.assert_close(conv.bias.grad, ref.bias.grad,
                                   atol=gt * max(1.0, ref.bias.grad.abs().max().item()), rtol=gt)


def test_dwconv_autocast_module():
    from realtime_semantic_segmentation_pytorch_amd.models.modules import DWConvBNAct

    torch.manual_seed(0)
    blk = DWConvBNAct(32, 32, 3, 1, 1, "relu").to(DEV)
    ops.convert_depthwise(blk)
    assert isinstance(blk[0], DepthwiseConv2d)
    x = torch.randn(4, 32, 24, 40, device=DEV).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = blk(x)
    assert y.dtype == torch.bfloat16
    y.float().sum().backward()
    assert blk[0].weight.grad is not None and blk[0].weight.grad.dtype == torch.float32
    with torch.no_grad():
        yr = F.relu(blk[1](F.conv2d(x, blk[0].weight, None, 1, 1, 1, 32)))
    torch.testing.assert_close(y.float(), yr, atol=5e-2, rtol=5e-2)


# ------------------------------------------------------ forward + BN statistics epilogue (K2)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("geom", [g for g in GEOMS if g[1] in (1, 2, 3, 4, 6)] + [
    (96, 1, (3, 3), 1, 1, (33, 17)),     # 12 channel vectors: grid rounded to a multiple of 3
    (768, 1, (3, 3), 1, 1, (8, 16)),     # 96 channel vectors (> 8 * 256 / 8 chunks of work)
    (48, 1, (3, 3), 1, 1, (200, 300)),   # many blocks
])
def test_dwconv_forward_stats_slab(dtype, geom):
    cin, mult, k, s, d, hw = geom
    torch.manual_seed(1)
    pad = tuple((kk - 1) // 2 * d for kk in k)
    cout = cin * mult
    w = torch.randn(cout, 1, *k, device=DEV)
    wt = w.reshape(cout, -1).t().contiguous()
    x = torch.randn(3, cin, *hw, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    y, part = torch.ops.rtseg.dw_conv_fwd_stats(x, wt, cout, k[0], k[1], s, s, pad[0], pad[1], d, d)
    y0 = torch.ops.rtseg.dw_conv_fwd(x, wt, None, cout, k[0], k[1], s, s, pad[0], pad[1], d, d)
    assert torch.equal(y, y0)
    assert part.dim() == 2 and part.shape[1] == 2 * cout and part.shape[0] > 0
    ref = F.conv2d(x.double(), w.double(), None, s, pad, d, cin)  # fp32 accumulators ~ fp64
    torch.testing.assert_close(part[:, :cout].double().sum(0), ref.sum((0, 2, 3)), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(part[:, cout:].double().sum(0), ref.square().sum((0, 2, 3)), rtol=1e-4, atol=1e-3)
    part2 = torch.ops.rtseg.dw_conv_fwd_stats(x, wt, cout, k[0], k[1], s, s, pad[0], pad[1], d, d)[1]
    assert torch.equal(part, part2)  # deterministic


@pytest.mark.parametrize("mult", [1, 6])
def test_dwconvbnact_training_uses_epilogue_stats(mult, monkeypatch):
    """DWConvBNAct (models/modules.py) in training: the forward takes the statistics from the
    depth-wise kernel (no separate BN statistics pass) and matches the PyTorch modules."""
    from realtime_semantic_segmentation_pytorch_amd.models.modules import DWConvBNAct

    torch.manual_seed(2)
    m = DWConvBNAct(32, 32 * mult, 3, 2 if mult > 1 else 1).to(DEV)
    ref = DWConvBNAct(32, 32 * mult, 3, 2 if mult > 1 else 1).to(DEV)
    ref.load_state_dict(m.state_dict())
    ops.convert_depthwise(m)
    ops.convert_batchnorm(m)
    calls = []
    orig = ops.dw_conv_bn_stats
    import realtime_semantic_segmentation_pytorch_amd.models.modules as M

    monkeypatch.setattr(M.ops, "dw_conv_bn_stats", lambda *a: calls.append(1) or orig(*a))
    x = torch.randn(4, 32, 24, 40, device=DEV).contiguous(memory_format=torch.channels_last)
    xr = x.clone().requires_grad_(True)
    x.requires_grad_(True)
    y = m(x)
    assert calls, "the depth-wise statistics path did not run"
    monkeypatch.setenv("RTSEG_DISABLE_HIP", "1")
    yr = ref(xr)
    monkeypatch.delenv("RTSEG_DISABLE_HIP")
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(m[1].running_mean, ref[1].running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(m[1].running_var, ref[1].running_var, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("mult,stride,act,bias", [(1, 1, "relu", False), (1, 2, "none", False), (6, 1, "none", False),
                                                 (6, 2, "relu6", False), (1, 1, "relu", True)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_dw_bn_eval_folded(mult, stride, act, bias, dtype):
    """Inference DWConvBNAct: the eval BN folded into the depth-wise weights / bias and the ReLU /
    ReLU6 applied in the kernel's store (ops.dw_conv_bn_eval), against conv -> BN -> act in fp32."""
    import torch.nn.functional as F

    from realtime_semantic_segmentation_pytorch_amd.models.modules import DWConvBNAct
    from realtime_semantic_segmentation_pytorch_amd.ops import dwconv as dw_mod

    assert ops.load()
    torch.manual_seed(mult + stride)
    cin = 32
    m = DWConvBNAct(cin, cin * mult, 3, stride, act_type=act)
    if bias:
        m[0] = torch.nn.Conv2d(cin, cin * mult, 3, stride, 1, groups=cin, bias=True)
    m = ops.convert_batchnorm(ops.convert_depthwise(m)).cuda().eval()
    with torch.no_grad():
        m[1].running_mean.uniform_(-0.3, 0.3)
        m[1].running_var.uniform_(0.5, 2.0)
        m[1].weight.uniform_(0.5, 1.5)
        m[1].bias.uniform_(-0.3, 0.3)
    x = torch.randn(2, cin, 33, 40, device="cuda").contiguous(memory_format=torch.channels_last)
    before = dw_mod.DW_BN_FOLDED[0]
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
        got = m(x)
    assert dw_mod.DW_BN_FOLDED[0] == before + 1
    xr = x.to(dtype).float()
    wr = m[0].weight.float() if dtype == torch.float32 else m[0].weight.to(dtype).float()
    with torch.no_grad():
        ref = F.conv2d(xr, wr, m[0].bias, stride, 1, 1, cin)
        ref = F.batch_norm(ref, m[1].running_mean, m[1].running_var, m[1].weight, m[1].bias, False, 0.0, m[1].eps)
    ref = ref.relu() if act == "relu" else ref.clamp(0, 6) if act == "relu6" else ref
    if dtype == torch.float32:
        torch.testing.assert_close(got.float(), ref, rtol=1e-4, atol=1e-4)
    else:
        torch.testing.assert_close(got.float(), ref, rtol=2 ** -7, atol=2e-3 * ref.abs().max().item())
