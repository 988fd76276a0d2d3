"""7 x 7 stem (csrc/kernels/conv_stem7.hip) against the fp32 PyTorch reference: raw conv and the
inference BN + activation epilogue, stride 1 / 2, odd output sizes, 16 / 32 / 48 / 64 outputs; and
the routed eval path of a ResNet stem (ops.conv_bn_act with an eval BN) matching the torch modules."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd import ops
from _tol import bf16_close, f32_close  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(got, ref, tol):
    err = (got.float() - ref.float()).abs().max().item() / max(ref.float().abs().max().item(), 1e-6)
    assert err < tol, err


@pytest.mark.parametrize("case", [(2, 64, 96, 2, 64), (1, 37, 130, 2, 32), (2, 40, 64, 1, 16), (3, 21, 34, 2, 48)])
@pytest.mark.parametrize("act", [None, 0, 1, 2])
def test_stem7_matches_fp32(case, act):
    assert ops.load()
    n, h, w, s, cout = case
    g = torch.Generator().manual_seed(3)
    x = torch.randn(n, 3, h, w, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cout, 3, 7, 7, generator=g) / 10).to(DEV, torch.bfloat16)
    wk = wt.permute(0, 2, 3, 1).contiguous()
    ss = None
    ref = F.conv2d(x.float(), wt.float(), None, s, 3)
    if act is not None:
        scale = torch.rand(cout, generator=g) + 0.5
        shift = torch.randn(cout, generator=g) * 0.2
        ss = torch.cat([scale, shift]).to(DEV)
        ref = ref * scale.to(DEV).view(1, -1, 1, 1) + shift.to(DEV).view(1, -1, 1, 1)
        ref = ref if act == 0 else torch.relu(ref) if act == 1 else F.relu6(ref)
    y = torch.ops.rtseg.conv_stem7(x, wk, [s, s], ss, act if act is not None else 0)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    bf16_close(y, ref)


def test_resnet_stem_eval_path_matches_torch(monkeypatch):
    """ops.conv_bn_act in bf16 inference routes the 7 x 7 stem + eval BN + ReLU to conv_stem7 when it
    wins its timing (forced here) and matches the stock modules."""
    from realtime_semantic_segmentation_pytorch_amd.ops import conv as conv_mod

    monkeypatch.setattr(conv_mod, "_choose", lambda key, cands: 0)
    torch.manual_seed(0)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(DEV)
    bn = nn.BatchNorm2d(64).to(DEV)
    with torch.no_grad():
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    conv.eval(), bn.eval()
    x = torch.randn(2, 3, 128, 256, device=DEV).contiguous(memory_format=torch.channels_last)
    called = []
    real = conv_mod._stem7_eval
    monkeypatch.setattr(conv_mod, "_stem7_eval", lambda *a: called.append(1) or real(*a))
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        got = ops.conv_bn_act(x, conv, bn, "relu")
        ref = torch.relu(bn(conv(x)))
    assert called
    _close(got, ref, 2e-2)
