"""CPU behaviour of the op wrappers: fallbacks equal the PyTorch formulation exactly."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.ops.optim import FusedAdam, FusedAdamW, FusedSGD, _dense


def _net():
    torch.manual_seed(0)
    return nn.Sequential(nn.Conv2d(3, 8, 3, bias=False), nn.BatchNorm2d(8), nn.ReLU(), nn.Flatten(),
                         nn.Linear(8 * 4 * 4, 3))


@pytest.mark.parametrize("cls,ref,kw", [
    (FusedSGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-4)),
    (FusedAdam, torch.optim.Adam, dict(lr=1e-3)),
    (FusedAdamW, torch.optim.AdamW, dict(lr=1e-3, weight_decay=0.01)),
])
def test_fused_optimizers_fall_back_to_torch_on_cpu(cls, ref, kw):
    a, b = _net(), _net()
    oa, ob = cls(a.parameters(), **kw), ref(b.parameters(), **kw)
    x = torch.randn(2, 3, 6, 6)
    for _ in range(3):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            m(x).square().mean().backward()
            o.step()
    assert not oa.last_step_fused
    for p, q in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(p, q)
    ob2 = ref(b.parameters(), **kw)
    ob2.load_state_dict(oa.state_dict())  # identical state layout


def test_dense_layouts():
    t = torch.randn(4, 3, 5, 5)
    assert _dense(t) and _dense(t.contiguous(memory_format=torch.channels_last))
    assert not _dense(t[:, :2]) and not _dense(t[..., ::2])


@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("residual", [False, True])
def test_conv_bn_act_cpu_matches_modules(train, residual):
    torch.manual_seed(1)
    conv, bn = nn.Conv2d(32, 16, 3, padding=1, bias=False), nn.BatchNorm2d(16)
    bn.running_mean.uniform_(-0.5, 0.5)
    bn.running_var.uniform_(0.5, 1.5)
    conv.train(train), bn.train(train)
    bn_ref = copy.deepcopy(bn)
    x = torch.randn(2, 32, 9, 11)
    res = torch.randn(2, 16, 9, 11) if residual else None
    y = ops.conv_bn_act(x, conv, bn, "relu", residual=res)
    r = bn_ref(conv(x))
    if residual:
        r = r + res
    torch.testing.assert_close(y, F.relu(r))
    torch.testing.assert_close(bn.running_mean, bn_ref.running_mean)


def test_depthwise_module_cpu_is_conv2d():
    torch.manual_seed(2)
    ref = nn.Conv2d(16, 96, 3, 2, 1, groups=16, bias=False)
    dw = copy.deepcopy(ref)
    ops.convert_depthwise(nn.Sequential(dw))
    assert isinstance(dw, ops.DepthwiseConv2d) and ops.depthwise_ok(ref)
    x = torch.randn(2, 16, 13, 17)
    torch.testing.assert_close(dw(x), ref(x))
    assert dw.state_dict().keys() == ref.state_dict().keys()


def test_kd_and_confmat_references_cpu():
    torch.manual_seed(3)
    s, t = torch.randn(2, 5, 4, 6), torch.randn(2, 5, 4, 6)
    got = ops.kd_kl_div(s, t, 4.0)
    want = F.kl_div(F.log_softmax(s / 4.0, 1), F.softmax(t / 4.0, 1)) * 16.0
    torch.testing.assert_close(got, want)
    y = torch.randint(0, 5, (2, 4, 6))
    y[0, 0, 0] = 255
    cm = ops.confusion_matrix(s, y, 5, 255)
    assert cm.sum().item() == y.numel() - 1 and cm.dtype == torch.int64


def test_ema_params_done_updates_only_buffers():
    from types import SimpleNamespace

    from realtime_semantic_segmentation_pytorch_amd.utils.optim import ModelEmaV2

    m = _net()
    ema = ModelEmaV2(SimpleNamespace(use_ema=True, total_itrs=10), m)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(1.0)
        m[1].running_mean.add_(1.0)
    before = [p.clone() for p in ema.ema.parameters()]
    ema.update(m, 5, params_done=True)
    for a, b in zip(before, ema.ema.parameters()):
        torch.testing.assert_close(a, b)  # parameters left to the fused optimizer
    torch.testing.assert_close(ema.ema[1].running_mean, torch.full((8,), 0.5))  # decay 0.5 lerp


def test_pooling_modules_cpu_match_torch():
    m = nn.Sequential(nn.MaxPool2d(3, 2, 1), nn.AvgPool2d(5, 2, 2), nn.AdaptiveAvgPool2d((2, 3)))
    ref = copy.deepcopy(m)
    ops.convert_pooling(m)
    assert isinstance(m[0], ops.MaxPool2d) and isinstance(m[1], ops.AvgPool2d)
    assert isinstance(m[2], ops.AdaptiveAvgPool2d)
    x = torch.randn(2, 4, 21, 30)
    torch.testing.assert_close(m(x), ref(x))
    assert m.state_dict().keys() == ref.state_dict().keys()


def test_detail_loss_cpu_is_reference():
    conv = nn.Conv2d(3, 1, 1, bias=False)
    labels = torch.randint(0, 19, (2, 32, 48))
    d = torch.randn(2, 1, 4, 6, requires_grad=True)
    got = ops.detail_loss(d, labels, conv, 0.1)
    want = ops.detail_loss_reference(d, labels, conv, 0.1)
    torch.testing.assert_close(got, want)
    got.backward()
    assert d.grad is not None and torch.isfinite(d.grad).all()


def test_colorize_reference_matches_pil_blend():
    import numpy as np
    from PIL import Image

    torch.manual_seed(5)
    logits = torch.randn(2, 19, 8, 12)
    cmap = torch.randint(0, 256, (19, 3), dtype=torch.uint8)
    img = torch.randint(0, 256, (2, 8, 12, 3), dtype=torch.uint8)
    cls, rgb, blend = ops.colorize(logits, cmap, img, 0.3)
    assert torch.equal(cls.long(), logits.argmax(1)) and torch.equal(rgb, cmap[logits.argmax(1)])
    for i in range(2):
        want = np.asarray(Image.blend(Image.fromarray(img[i].numpy()), Image.fromarray(rgb[i].numpy()), 0.3))
        assert np.array_equal(blend[i].numpy(), want)


@pytest.mark.parametrize("k,axis,d,cin,cout", [(3, 0, 2, 4, 4), (3, 1, 16, 8, 8), (5, 0, 3, 16, 8), (3, 1, 4, 4, 16)])
def test_tap_conv_matches_conv2d_cpu(k, axis, d, cin, cout):
    """ops/tapconv.py: per-tap GEMM formulation == F.conv2d (values and gradients)."""
    import torch.nn.functional as F
    from realtime_semantic_segmentation_pytorch_amd.ops import tap_conv2d, tapconv_ok

    torch.manual_seed(0)
    ks = (k, 1) if axis == 0 else (1, k)
    pad = (d * (k - 1) // 2, 0) if axis == 0 else (0, d * (k - 1) // 2)
    conv = torch.nn.Conv2d(cin, cout, ks, padding=pad, dilation=(d, 1) if axis == 0 else (1, d), bias=True).double()
    assert tapconv_ok(conv)
    x = torch.randn(2, cin, 37, 41, dtype=torch.float64).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    ref = F.conv2d(x, conv.weight, conv.bias, 1, pad, conv.dilation)
    got = tap_conv2d(x, conv.weight, conv.bias, d, axis)
    torch.testing.assert_close(got, ref)
    g = torch.randn_like(ref)
    gx_ref, gw_ref = torch.autograd.grad(ref, (x, conv.weight), g)
    gx, gw = torch.autograd.grad(got, (x, conv.weight), g)
    torch.testing.assert_close(gx, gx_ref)
    torch.testing.assert_close(gw, gw_ref)


def test_tap_conv_converted_only_in_cfpnet_like_layers_cpu():
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.models import get_model
    from realtime_semantic_segmentation_pytorch_amd.ops import TapConv2d

    c = BaseConfig()
    c.model, c.num_class = "cfpnet", 19
    m = get_model(c)
    n = sum(type(x) is TapConv2d for x in m.modules())
    assert n > 0
    keys = set(m.state_dict())
    assert any(k.endswith("block1.0.0.weight") for k in keys)


@pytest.mark.parametrize("hw,d,groups", [((20, 24), (2, 2), 4), ((19, 23), (3, 5), 2), ((17, 16), (14, 14), 8)])
def test_dilated_group_conv_space_to_batch_cpu(hw, d, groups):
    """ops/dilated.py: space-to-batch grouped conv == dilated grouped F.conv2d (values, grads)."""
    import torch.nn.functional as F
    from realtime_semantic_segmentation_pytorch_amd.ops import dilated_group_conv2d, dilated_group_ok

    torch.manual_seed(0)
    conv = torch.nn.Conv2d(32, 32, 3, padding=d, dilation=d, groups=groups, bias=True).double()
    assert dilated_group_ok(conv)
    x = torch.randn(2, 32, *hw, dtype=torch.float64).requires_grad_(True)
    ref = F.conv2d(x, conv.weight, conv.bias, 1, d, d, groups)
    got = dilated_group_conv2d(x, conv.weight, conv.bias, d, groups)
    torch.testing.assert_close(got, ref)
    g = torch.randn_like(ref)
    r = torch.autograd.grad(ref, (x, conv.weight, conv.bias), g)
    q = torch.autograd.grad(got, (x, conv.weight, conv.bias), g)
    for a, b in zip(q, r):
        torch.testing.assert_close(a, b)


@pytest.mark.parametrize("hw,k,s,p,d", [
    ((8, 16), (3, 3), (1, 1), (14, 14), (14, 14)),   # RegSeg DBlock at 1/16 of 128x256
    ((16, 32), (3, 1), (1, 1), (17, 0), (17, 1)),    # LEDNet (3, 1), dilation 17
    ((8, 16), (3, 3), (1, 1), (12, 12), (12, 12)),   # LiteSeg / ASPP branch
    ((5, 7), (5, 3), (2, 1), (6, 1), (3, 1)),        # strided, asymmetric leftovers
    ((1, 2), (3, 3), (1, 1), (1, 1), (1, 1)),        # 3x3 on a 1x2 map
    ((3, 9), (7, 7), (1, 2), (9, 3), (2, 1)),
    ((20, 24), (3, 3), (1, 1), (2, 2), (2, 2)),      # nothing dead: plain F.conv2d
])
def test_pruned_conv_drops_only_dead_taps_cpu(hw, k, s, p, d):
    """ops/dilated.py: dead-tap pruning is exact (values and all three gradients; the dropped
    taps' weight gradient is 0)."""
    import torch.nn.functional as F
    from realtime_semantic_segmentation_pytorch_amd.ops import has_dead_taps, pruned_conv2d

    torch.manual_seed(0)
    w = torch.randn(6, 4, *k, dtype=torch.float64, requires_grad=True)
    b = torch.randn(6, dtype=torch.float64, requires_grad=True)
    x = torch.randn(2, 4, *hw, dtype=torch.float64, requires_grad=True)
    ref = F.conv2d(x, w, b, s, p, d)
    got = pruned_conv2d(x, w, b, s, p, d, 1)
    assert got.shape == ref.shape
    torch.testing.assert_close(got, ref)
    g = torch.randn_like(ref)
    for a, r in zip(torch.autograd.grad(got, (x, w, b), g), torch.autograd.grad(ref, (x, w, b), g)):
        torch.testing.assert_close(a, r)
    assert has_dead_taps(hw, k, s, p, d) == (hw != (20, 24))


@pytest.mark.parametrize("hw,d", [((8, 16), (14, 14)), ((8, 16), (4, 14)), ((3, 3), (5, 5)), ((9, 9), (2, 3))])
def test_dilated_group_conv_prunes_then_space_to_batch_cpu(hw, d):
    import torch.nn.functional as F
    from realtime_semantic_segmentation_pytorch_amd.ops.dilated import dilated_group_pruned

    torch.manual_seed(0)
    w = torch.randn(32, 4, 3, 3, dtype=torch.float64, requires_grad=True)
    x = torch.randn(2, 32, *hw, dtype=torch.float64, requires_grad=True)
    ref = F.conv2d(x, w, None, 1, d, d, 8)
    got = dilated_group_pruned(x, w, None, d, 8)
    torch.testing.assert_close(got, ref)
    g = torch.randn_like(ref)
    for a, r in zip(torch.autograd.grad(got, (x, w), g), torch.autograd.grad(ref, (x, w), g)):
        torch.testing.assert_close(a, r)


def test_pruned_convs_converted_in_zoo_cpu():
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.models import get_model
    from realtime_semantic_segmentation_pytorch_amd.ops import PrunedConv2d

    c = BaseConfig()
    c.model, c.num_class = "lednet", 19
    m = get_model(c)
    assert not any(type(x) is torch.nn.Conv2d and max(x.kernel_size) > 1 for x in m.modules())
    assert any(type(x) is PrunedConv2d and max(x.dilation) > 1 for x in m.modules())


def test_dilated_group_conv_converted_in_regseg_cpu():
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.models import get_model
    from realtime_semantic_segmentation_pytorch_amd.ops import DilatedGroupConv2d

    c = BaseConfig()
    c.model, c.num_class = "regseg", 19
    assert any(type(x) is DilatedGroupConv2d for x in get_model(c).modules())


def test_convert_activations_keeps_state_and_cpu_semantics():
    import torch.nn as nn

    from realtime_semantic_segmentation_pytorch_amd.ops import act as A

    net = nn.Sequential(nn.Conv2d(3, 8, 3), nn.PReLU(8), nn.ELU(), nn.Hardswish(), nn.SiLU(), nn.ReLU6())
    ref = {k: v.clone() for k, v in net.state_dict().items()}
    x = torch.randn(2, 3, 9, 9)
    y0 = net(x)
    A.convert_activations(net)
    assert type(net[1]).__name__ == "HipPReLU" and isinstance(net[1], nn.PReLU)
    assert type(net[5]) is nn.ReLU6  # ReLU6 stays: the BN / conv epilogues fuse it
    assert net.state_dict().keys() == ref.keys()
    assert torch.equal(net(x), y0)  # CPU tensors run the module's own forward


def test_conv_tuning_db_roundtrip(tmp_path, monkeypatch):
    """Per-shape conv winners persist across processes (ops/conv.py tuning database) and are
    only reused on the architecture that measured them."""
    import json

    from realtime_semantic_segmentation_pytorch_amd.ops import conv as C

    out = tmp_path / "db.json"
    monkeypatch.setenv("RTSEG_TUNE_DB_OUT", str(out))
    monkeypatch.setenv("RTSEG_TUNE_DB", str(out))
    monkeypatch.setattr(C, "_DB", None)
    key = ("dgrad", (32, 64, 256, 512), 64, 3, 3, (1, 1), (1, 1), (1, 1))
    C._db_record(key, "igemm")
    monkeypatch.setattr(C, "_DB", None)
    assert C._tune_db()[repr(key)] == "igemm"
    data = json.loads(out.read_text())
    data["arch"] = "gfx000"  # another architecture's measurements are ignored
    out.write_text(json.dumps(data))
    monkeypatch.setattr(C, "_DB", None)
    assert C._tune_db() == {}
    monkeypatch.setattr(C, "_DB", None)


@pytest.mark.parametrize("groups,cout,cg,k", [(8, 128, 16, 3), (3, 48, 16, 3), (4, 8, 2, 1)])
def test_block_diagonal_grouped_conv_identity(groups, cout, cg, k):
    """The grouped-conv route (ops/conv.py grouped_as_dense): a dense conv of the block-diagonal
    weight is the grouped conv, and the weight gradient flows back to the grouped weight."""
    from realtime_semantic_segmentation_pytorch_amd.ops.conv import block_diagonal

    torch.manual_seed(0)
    x = torch.randn(2, cg * groups, 9, 11, dtype=torch.float64)
    w = torch.randn(cout, cg, k, k, dtype=torch.float64, requires_grad=True)
    w2 = w.detach().clone().requires_grad_(True)
    y = F.conv2d(x, block_diagonal(w, groups), None, 1, k // 2, 1, 1)
    ref = F.conv2d(x, w2, None, 1, k // 2, 1, groups)
    torch.testing.assert_close(y, ref)
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g)
    torch.testing.assert_close(w.grad, w2.grad)


def test_cat_bn_act_cpu_matches_cat_then_bn():
    """ops.cat_bn_act on the CPU: the concat + BatchNorm (+ ReLU / PReLU module) of the reference
    formulation, including the running statistics (GPU kernels: tests/test_concat_gpu.py)."""
    import copy

    from realtime_semantic_segmentation_pytorch_amd import ops
    from realtime_semantic_segmentation_pytorch_amd.models.modules import Activation

    torch.manual_seed(0)
    parts = [torch.randn(2, 8, 5, 7), torch.randn(2, 16, 5, 7) + 1.0]
    for act in ("relu", "prelu"):
        bn = torch.nn.BatchNorm2d(24).train()
        actm = Activation(act)
        b2, a2 = copy.deepcopy(bn), copy.deepcopy(actm)
        y = ops.cat_bn_act(parts, bn, actm, act_module=actm)
        ref = a2(b2(torch.cat(parts, dim=1)))
        torch.testing.assert_close(y, ref)
        torch.testing.assert_close(bn.running_mean, b2.running_mean)
        torch.testing.assert_close(bn.running_var, b2.running_var)


def test_concat_sink_pooled_part_cpu_fallback():
    """ConcatSink.max_pool off the GPU: a plain pooled tensor (cast to the concat dtype when asked),
    and cat() is torch.cat -- the reference's StemBlock / InitialBlock semantics."""
    x = torch.randn(2, 16, 9, 14)
    sink = ops.ConcatSink([16, 16])
    p = sink.max_pool(1, x, 3, 2, 1)
    assert isinstance(p, torch.Tensor)
    torch.testing.assert_close(p, F.max_pool2d(x, 3, 2, 1))
    y = torch.randn(2, 16, 5, 7)
    torch.testing.assert_close(sink.cat([y, p]), torch.cat([y, p], 1))
    pb = ops.ConcatSink([16, 16]).max_pool(1, x, 3, 2, 1, dtype=torch.bfloat16)
    assert pb.dtype == torch.bfloat16
    torch.testing.assert_close(pb, F.max_pool2d(x, 3, 2, 1).to(torch.bfloat16))


def test_stem_blocks_cpu_match_plain_cat():
    """BiSeNetV2's StemBlock and the ENet-family InitialBlock (concat sinks on the GPU) equal the
    reference formulation -- conv_last(cat(left, maxpool)) / cat(conv, maxpool) -- on the CPU."""
    from realtime_semantic_segmentation_pytorch_amd.models.bisenetv2 import StemBlock
    from realtime_semantic_segmentation_pytorch_amd.models.enet import InitialBlock

    torch.manual_seed(0)
    stem = StemBlock(3, 16).eval()
    x = torch.randn(2, 3, 32, 48)
    with torch.no_grad():
        s = stem.conv_init(x)
        want = stem.conv_last(torch.cat([stem.left_branch(s), stem.right_branch(s)], 1))
        torch.testing.assert_close(stem(x), want)
        ib = InitialBlock(16, 64, "relu").eval()
        z = torch.randn(2, 16, 20, 30)
        torch.testing.assert_close(ib(z), torch.cat([ib.conv(z), ib.pool(z)], 1))
