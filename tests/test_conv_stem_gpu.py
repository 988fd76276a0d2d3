"""3-channel stem conv (csrc/kernels/conv_stem.hip) vs fp32 PyTorch on the same bf16 operands:
forward (+ BN-statistics slab) and weight gradient of 3x3 / pad-1 convs with Cin = 3, stride 1
and 2, Cout 16 / 32 / 48 / 64 -- partial tiles (Ho % 8, Wo % 64), fewer tiles than blocks and
many tiles per block, both parameter layouts; deterministic.  Reference layer: DDRNet's conv1
(reference models/ddrnet.py:27-29), the stems of the STDC / BiSeNet / ResNet families.
Also the twin conv node of downsampling residual blocks (ops/conv.py _TwinConvFn, reference
models/ddrnet.py:168-219) against the two separate conv nodes."""
import pytest
import torch
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd import ops
from _tol import bf16_close, f32_close  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (n, h, w, cout, stride); w even
GEOMS = [(2, 17, 70, 64, 2), (1, 9, 130, 32, 1), (3, 33, 66, 16, 2), (2, 20, 128, 48, 1),
         (8, 256, 512, 64, 2), (1, 5, 6, 64, 2)]


@pytest.fixture(autouse=True)
def _lib():
    assert ops.load(), "HIP extension must load on the GPU box"


def _t(shape, g, scale=1.0):
    return (torch.randn(shape, generator=g) * scale).to(DEV, torch.bfloat16)


def _close(got, ref, tol):
    torch.testing.assert_close(got.float(), ref, atol=tol * ref.abs().max().item() + 1e-6, rtol=tol)


@pytest.mark.parametrize("geom", GEOMS)
def test_stem_forward_and_stats(geom):
    n, h, w, cout, s = geom
    g = torch.Generator().manual_seed(0)
    x = _t((n, 3, h, w), g).contiguous(memory_format=torch.channels_last)
    wt = _t((cout, 3, 3, 3), g, 0.2)
    wk = wt.permute(0, 2, 3, 1).contiguous()
    y, part = torch.ops.rtseg.conv_stem(x, wk, [s, s], [1, 1], [1, 1], True)
    ref = F.conv2d(x.float(), wt.float(), None, s, 1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    bf16_close(y, ref)
    rf = ref.double()  # statistics of the fp32 accumulators
    torch.testing.assert_close(part[:, :cout].double().sum(0), rf.sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[:, cout:].double().sum(0), rf.square().sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    y1, p1 = torch.ops.rtseg.conv_stem(x, wk, [s, s], [1, 1], [1, 1], True)
    assert torch.equal(y1, y) and torch.equal(p1, part)
    y2, p2 = torch.ops.rtseg.conv_stem(x, wk, [s, s], [1, 1], [1, 1], False)
    assert torch.equal(y2, y) and (p2 is None or p2.numel() == 0)


@pytest.mark.parametrize("geom", GEOMS)
@pytest.mark.parametrize("channels_last", [False, True])
def test_stem_wgrad(geom, channels_last):
    n, h, w, cout, s = geom
    g = torch.Generator().manual_seed(3)
    cl = dict(memory_format=torch.channels_last)
    x = _t((n, 3, h, w), g).contiguous(**cl)
    ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
    dy = _t((n, cout, ho, wo), g).contiguous(**cl)
    dw = torch.ops.rtseg.conv_stem_wgrad(x, dy, 3, 3, [s, s], [1, 1], [1, 1], channels_last)
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, 3, 3, 3), dy.float(), s, 1, 1)
    assert dw.shape == ref.shape and dw.dtype == torch.float32
    assert dw.is_contiguous(memory_format=torch.channels_last) == channels_last
    f32_close(dw, ref)
    assert torch.equal(torch.ops.rtseg.conv_stem_wgrad(x, dy, 3, 3, [s, s], [1, 1], [1, 1], channels_last), dw)


def test_stem_rejects_other_shapes():
    g = torch.Generator().manual_seed(1)
    x = _t((1, 3, 8, 33), g).contiguous(memory_format=torch.channels_last)  # odd width
    with pytest.raises(RuntimeError, match="conv_stem"):
        torch.ops.rtseg.conv_stem(x, _t((64, 3, 3, 3), g), [2, 2], [1, 1], [1, 1], False)
    x = _t((1, 3, 8, 32), g).contiguous(memory_format=torch.channels_last)
    with pytest.raises(RuntimeError, match="conv_stem"):  # Cout not a multiple of 16
        torch.ops.rtseg.conv_stem(x, _t((24, 3, 3, 3), g), [2, 2], [1, 1], [1, 1], False)


def test_stem_routed_training_step(monkeypatch):
    """DDRNet's conv1 (ConvBNAct 3 -> 64, stride 2) with conv_stem forced vs MIOpen: outputs, BN
    statistics and weight gradients agree up to bf16 rounding, and the routing called the kernels."""
    from realtime_semantic_segmentation_pytorch_amd.models.modules import ConvBNAct
    from realtime_semantic_segmentation_pytorch_amd.ops import conv as conv_mod

    torch.manual_seed(0)
    net = ops.convert_batchnorm(ConvBNAct(3, 64, 3, 2)).to(DEV).to(memory_format=torch.channels_last).train()
    x = torch.randn(2, 3, 48, 132, device=DEV).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(2, 64, 24, 66, device=DEV)
    calls = []

    class _Spy:
        def __getattr__(self, name):
            calls[-1].add(name)
            return getattr(torch.ops.rtseg, name)

    monkeypatch.setattr(conv_mod, "ops", lambda: spy)
    spy = _Spy()
    res = []
    for mode in ("1", "0"):
        monkeypatch.setenv("RTSEG_CONV_STEM", mode)
        if mode == "1":  # the first candidate, no timing
            monkeypatch.setenv("RTSEG_CONV_MFMA", "1")
        else:
            monkeypatch.delenv("RTSEG_CONV_MFMA", raising=False)
        calls.append(set())
        net.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = net(x)
        (y.float() * gy).sum().backward()
        res.append((y.float().detach(), {n: p.grad.float().clone() for n, p in net.named_parameters()}))
    (y0, gp0), (y1, gp1) = res

    def rel(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()

    assert rel(y0, y1) < 1e-2
    for n, g in gp1.items():
        assert rel(gp0[n], g) < 2e-2, n
    # the stem's BN hands its dx pass to the stem weight gradient (conv_stem_wgrad_bn)
    assert "conv_stem" in calls[0] and calls[0] & {"conv_stem_wgrad", "conv_stem_wgrad_bn"}, calls[0]
    assert not {"conv_stem", "conv_stem_wgrad", "conv_stem_wgrad_bn"} & calls[1], calls[1]


@pytest.mark.parametrize("block", ["RB", "RBB"])
def test_twin_conv_downsample_block(monkeypatch, block):
    """A downsampling DDRNet block with conv1 + projection shortcut in one autograd node
    (ops.twin_conv_bn_stats) vs the two separate conv nodes: identical forward, input and
    parameter gradients up to bf16 rounding; the twin path leaves no accumulation add."""
    from realtime_semantic_segmentation_pytorch_amd.models import ddrnet

    torch.manual_seed(0)
    cls = getattr(ddrnet, block)
    net = ops.convert_batchnorm(cls(64, 128, 2)).to(DEV).to(memory_format=torch.channels_last).train()
    x0 = torch.randn(2, 64, 32, 96, device=DEV).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(2, 128, 16, 48, device=DEV)
    res = []
    for twin in ("1", "0"):
        monkeypatch.setenv("RTSEG_TWIN_CONV", twin)
        net.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = net(x)
        (y.float() * gy).sum().backward()
        res.append((y.float().detach(), x.grad.float().clone(),
                    {n: p.grad.float().clone() for n, p in net.named_parameters()}))
    (y0, gx0, gp0), (y1, gx1, gp1) = res

    def rel(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()

    assert rel(y0, y1) < 1e-2
    assert rel(gx0, gx1) < 2e-2
    for n, g in gp1.items():
        assert rel(gp0[n], g) < 3e-2, n


def test_twin_conv_node_in_graph(monkeypatch):
    """The twin node really is on the training path of a downsampling RB."""
    from realtime_semantic_segmentation_pytorch_amd.models.ddrnet import RB

    monkeypatch.setenv("RTSEG_TWIN_CONV", "1")
    net = ops.convert_batchnorm(RB(64, 128, 2)).to(DEV).to(memory_format=torch.channels_last).train()
    x = torch.randn(1, 64, 16, 64, device=DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = net(x)
    seen, stack, names = set(), [y.grad_fn], set()
    while stack:
        fn = stack.pop()
        if fn is None or id(fn) in seen:
            continue
        seen.add(id(fn))
        names.add(type(fn).__name__)
        stack.extend(f for f, _ in fn.next_functions)
    assert any("TwinConvFn" in n for n in names), names


@pytest.mark.parametrize("cout,stride,bias", [(8, 2, False), (3, 1, True), (32, 2, False), (19, 1, True)])
def test_stem_inference_path(cout, stride, bias):
    """bf16 inference of a 3-channel stem conv (ops.conv_forward -> conv_stem.hip, weight zero-padded
    to 16 channels and cached) == F.conv2d on the same bf16 operands in fp32, for output counts the
    kernel does not tile natively (DFANet's 3 -> 8, ESPNetv2's 3 -> 3)."""
    from realtime_semantic_segmentation_pytorch_amd.ops import conv as conv_mod

    g = torch.Generator().manual_seed(cout)
    conv = torch.nn.Conv2d(3, cout, 3, stride, 1, bias=bias).to(DEV).eval()
    conv.__class__ = ops.RoutedConv2d if not bias else ops.PrunedConv2d
    x = torch.randn(2, 3, 34, 66, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    assert conv_mod.stem_infer_ok(conv, x)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops.conv_forward(x, conv)
        y2 = ops.conv_forward(x, conv)  # the cached weight
    xb, wb = x.to(torch.bfloat16).float(), conv.weight.to(torch.bfloat16).float()
    ref = F.conv2d(xb, wb, None, stride, 1)
    if bias:
        ref = ref + conv.bias.to(torch.bfloat16).float().view(1, -1, 1, 1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    bf16_close(y, ref)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("act", ["relu", "none", "relu6"])
@pytest.mark.parametrize("second_consumer", [False, True])
@pytest.mark.parametrize("cout", [64, 32])
def test_stem_bn_backward_fused(monkeypatch, act, second_consumer, cout):
    """The BN after a stem conv hands its backward dx pass to the stem's weight gradient
    (ops/bn.py _stem_handoff -> conv_stem_wgrad_bn): conv weight, BN weight / bias gradients equal
    the unfused path (RTSEG_STEM_BN_FUSE off) up to bf16 rounding of dx; with a second consumer
    of the conv output the fallback (materialised dx + the other gradient) is taken."""
    from realtime_semantic_segmentation_pytorch_amd.ops import bn as bn_mod
    from realtime_semantic_segmentation_pytorch_amd.ops import conv as conv_mod

    monkeypatch.setenv("RTSEG_CONV_MFMA", "1")  # the stem kernel in the forward, no timing
    torch.manual_seed(1)
    conv = torch.nn.Conv2d(3, cout, 3, 2, 1, bias=False).to(DEV)
    conv.__class__ = ops.PrunedConv2d
    bn = ops.convert_batchnorm(torch.nn.Sequential(torch.nn.BatchNorm2d(cout)))[0].to(DEV).train()
    x = torch.randn(2, 3, 40, 130, device=DEV).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(2, cout, 20, 65, device=DEV)
    res = []
    for fuse in (True, False):
        monkeypatch.setattr(conv_mod, "_STEM_BN_FUSE", fuse)
        for p in (conv.weight, bn.weight, bn.bias):
            p.grad = None
        n0 = bn_mod.STEM_HANDOFFS[0]
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y, part = ops.conv_bn_stats(x, conv)
            out = ops.bn_act(y, bn, act, part=part)
        loss = (out.float() * gy).sum()
        if second_consumer:
            loss = loss + 0.25 * (y.float() * gy.flip(0)).sum()
        loss.backward()
        assert (bn_mod.STEM_HANDOFFS[0] - n0) == (1 if fuse else 0)
        res.append([t.grad.float().clone() for t in (conv.weight, bn.weight, bn.bias)])

    def rel(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()

    for a, b, name in zip(res[0], res[1], ("conv.weight", "bn.weight", "bn.bias")):
        assert rel(a, b) < 1e-2, (name, rel(a, b))


@pytest.mark.parametrize("geom", [(2, 17, 70, 64, 2), (1, 9, 130, 32, 1), (3, 33, 66, 16, 2)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_stem_bn_act_epilogue(geom, act):
    """conv_stem_bn_act: act(conv(x) * scale + shift) from the fp32 accumulators vs fp32 PyTorch."""
    n, h, w, cout, s = geom
    g = torch.Generator().manual_seed(4)
    x = _t((n, 3, h, w), g).contiguous(memory_format=torch.channels_last)
    wt = _t((cout, 3, 3, 3), g, 0.2)
    ss = torch.cat([torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g)]).to(DEV)
    y = torch.ops.rtseg.conv_stem_bn_act(x, wt.permute(0, 2, 3, 1).contiguous(), [s, s], [1, 1], [1, 1], ss, act)
    ref = F.conv2d(x.float(), wt.float(), None, s, 1) * ss[:cout].view(1, -1, 1, 1) + ss[cout:].view(1, -1, 1, 1)
    ref = ref.relu() if act == 1 else ref.clamp(0, 6) if act == 2 else ref
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    bf16_close(y, ref)


@pytest.mark.parametrize("no_store", [True, False])
@pytest.mark.parametrize("act", ["relu", "none"])
def test_stem_bn_forward_recompute(monkeypatch, act, no_store):
    """A training stem ConvBNAct: the BN's forward apply recomputed from the image
    (conv_stem_bn_act, ops/bn.py) vs the apply over the stored conv output -- outputs, BN running
    statistics and gradients agree to bf16 rounding, and the recompute really ran."""
    from realtime_semantic_segmentation_pytorch_amd.models.modules import ConvBNAct
    from realtime_semantic_segmentation_pytorch_amd.ops import bn as bn_mod
    from realtime_semantic_segmentation_pytorch_amd.ops import conv as conv_mod

    monkeypatch.setattr(conv_mod, "_STEM_NO_STORE", no_store)  # stats-only launch + wgrad recompute
    torch.manual_seed(0)
    net0 = ops.convert_batchnorm(ConvBNAct(3, 32, 3, 2, act_type=act)).to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(2, 3, 40, 132, device=DEV).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(2, 32, 20, 66, device=DEV)
    res = []
    for on in (True, False):
        import copy

        net = copy.deepcopy(net0).train()
        monkeypatch.setattr(bn_mod, "_STEM_BN_RECOMPUTE", on)
        before = bn_mod.STEM_RECOMPUTES[0]
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = net(x)
        seen, stack, stored = set(), [y.grad_fn], []
        while stack:  # the stem conv node: its statistics launch stored no output when recomputing
            fn = stack.pop()
            if fn is None or id(fn) in seen:
                continue
            seen.add(id(fn))
            if hasattr(fn, "y_stored"):
                stored.append(fn.y_stored)
            stack.extend(f for f, _ in fn.next_functions)
        assert stored == [not (on and no_store)], stored
        (y.float() * gy).sum().backward()
        assert (bn_mod.STEM_RECOMPUTES[0] > before) == on
        bn = [m for m in net.modules() if isinstance(m, torch.nn.BatchNorm2d)][0]
        res.append((y.float().detach(), {n: p.grad.float().clone() for n, p in net.named_parameters()},
                    bn.running_mean.clone(), bn.running_var.clone()))
    (y0, g0, m0, v0), (y1, g1, m1, v1) = res

    def rel(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()

    assert rel(y0, y1) < 1e-2
    torch.testing.assert_close(m0, m1)
    torch.testing.assert_close(v0, v1)
    for n_, g_ in g1.items():
        assert rel(g0[n_], g_) < 2e-2, n_


@pytest.mark.parametrize("geom", [(2, 17, 70, 64, 2), (1, 9, 130, 32, 1), (3, 33, 66, 16, 2)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_stem_bn_backward_sums_recompute(geom, act):
    """conv_stem_bn_sums (the stem BN's backward reduction with the conv output recomputed from the
    image) vs the same sums over the stored bf16 conv output in fp64: sum g' and sum g' (x - mean),
    g' = dy masked by act'(x * scale + shift)."""
    n, h, w, cout, s = geom
    g = torch.Generator().manual_seed(6)
    x = _t((n, 3, h, w), g).contiguous(memory_format=torch.channels_last)
    wt = _t((cout, 3, 3, 3), g, 0.2)
    wk = wt.permute(0, 2, 3, 1).contiguous()
    y, _ = torch.ops.rtseg.conv_stem(x, wk, [s, s], [1, 1], [1, 1], False)  # the stored conv output
    dy = _t(y.shape, g).contiguous(memory_format=torch.channels_last)
    mean = torch.randn(cout, generator=g) * 0.1
    mi = torch.cat([mean, torch.rand(cout, generator=g) + 0.5]).to(DEV)
    ss = torch.cat([torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g) * 0.3]).to(DEV)
    slab = torch.ops.rtseg.conv_stem_bn_sums(x, wk, [s, s], [1, 1], [1, 1], dy, mi, ss, act)
    got = slab.double().sum(0)
    xd, gd = y.double(), dy.double()
    z = xd * ss[:cout].double().view(1, -1, 1, 1) + ss[cout:].double().view(1, -1, 1, 1)
    live = torch.ones_like(z, dtype=torch.bool) if act == 0 else (z > 0) if act == 1 else (z > 0) & (z < 6)
    gm = torch.where(live, gd, torch.zeros_like(gd))
    ref_s = gm.sum((0, 2, 3))
    ref_q = (gm * (xd - mi[:cout].double().view(1, -1, 1, 1))).sum((0, 2, 3))
    scale = gd.abs().sum((0, 2, 3)).max().item()
    torch.testing.assert_close(got[:cout], ref_s, atol=1e-4 * scale, rtol=1e-4)
    torch.testing.assert_close(got[cout:], ref_q, atol=1e-4 * scale * xd.abs().max().item(), rtol=1e-4)


@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("act", ["relu", "none"])
def test_stem_eval_bn_in_epilogue(stride, act):
    """ops.conv_bn_act in bf16 inference on a 3-channel 3 x 3 stem: the eval BN (+ ReLU) runs in
    conv_stem.hip's epilogue (one pass) and matches fp32 BN(conv) of the bf16 operands."""
    import torch.nn as nn

    assert ops.load()
    torch.manual_seed(3)
    conv = nn.Conv2d(3, 32, 3, stride, 1, bias=False).to(DEV)
    bn = nn.BatchNorm2d(32).to(DEV)
    with torch.no_grad():
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    conv.eval(), bn.eval()
    x = torch.randn(2, 3, 66, 130, device=DEV).contiguous(memory_format=torch.channels_last)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        got = ops.conv_bn_act(x, conv, bn, act)
    xb, wb = x.to(torch.bfloat16).float(), conv.weight.to(torch.bfloat16).float()
    with torch.no_grad():
        ref = bn(F.conv2d(xb, wb, None, stride, 1))
    ref = ref.relu() if act == "relu" else ref
    assert got.dtype == torch.bfloat16 and got.is_contiguous(memory_format=torch.channels_last)
    bf16_close(got, ref)
