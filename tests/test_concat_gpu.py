"""Concat elimination (ops/concat.py): the BN kernels' concat-buffer store and the
strided gradient slice they read, against the dense formulation, and STDC modules (stride 1 and
2) trained through the sink against the same modules on plain ``torch.cat``."""
import copy

import pytest
import torch

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.ops import concat as concat_mod

pytestmark = pytest.mark.gpu

CL = dict(memory_format=torch.channels_last)


@pytest.fixture(autouse=True)
def _hip():
    assert ops.load()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("mask_bits", [False, True])
def test_bn_kernels_concat_slice(dtype, mask_bits):
    """bn_apply(out2) stores y into the slice; bn_backward(grad2) == bn_backward(dy + slice)."""
    g = torch.Generator().manual_seed(3)
    n, c, h, w, total, off = 2, 64, 9, 17, 160, 32
    x = torch.randn(n, c, h, w, generator=g).cuda().to(dtype).contiguous(**CL)
    res = torch.randn(n, c, h, w, generator=g).cuda().to(dtype).contiguous(**CL) if mask_bits else None
    wt, b = torch.rand(c).cuda() + 0.5, torch.randn(c).cuda()
    mi, ss, sums = torch.ops.rtseg.bn_stats_finalize(x, wt, b, None, None, None, 0.1, 1e-5)
    buf = torch.zeros(n, total, h, w, dtype=dtype, device="cuda").contiguous(**CL)
    sl = buf[:, off:off + c]
    if mask_bits:
        y, bits = torch.ops.rtseg.bn_apply_bits(x, ss, res, 1, sl)
        y0, bits0 = torch.ops.rtseg.bn_apply_bits(x, ss, res, 1)
        assert torch.equal(bits, bits0)
        ysave, mask = bits, 3
    else:
        y = torch.ops.rtseg.bn_apply(x, ss, None, 1, sl)
        y0 = torch.ops.rtseg.bn_apply(x, ss, None, 1)
        ysave, mask = None, 2
    assert torch.equal(y, y0) and torch.equal(sl, y)
    assert buf[:, :off].abs().sum() == 0 and buf[:, off + c:].abs().sum() == 0
    dbuf = torch.randn(n, total, h, w, generator=g).cuda().to(dtype).contiguous(**CL)
    d2 = dbuf[:, off:off + c]
    dy = torch.randn(n, c, h, w, generator=g).cuda().to(dtype).contiguous(**CL)
    # reference: the dense fp32 formulation on the same (exactly representable) values -- the
    # kernels add the slice in fp32 as well, so the parameter gradients agree to fp32 rounding
    x32 = x.float().contiguous(**CL)
    ysave32 = ysave
    if mask_bits:  # the fp32 kernels' bit mask has one byte per 4 channels (bf16: per 8)
        ysave32 = torch.ops.rtseg.bn_apply_bits(x32, ss, res.float().contiguous(**CL), 1)[1]
    for dense in (dy, None):
        tot = (d2.float() + (dense.float() if dense is not None else 0)).contiguous(**CL)
        want = torch.ops.rtseg.bn_backward(tot, x32, ysave32, None, sums, mi, ss, wt, 1, mask, mask_bits, True, True,
                                           None)
        got = torch.ops.rtseg.bn_backward(dense, x, ysave, None, sums, mi, ss, wt, 1, mask, mask_bits, True, True,
                                          None, d2)
        out_tol = 1e-5 if dtype == torch.float32 else 1e-2  # dx / dres are stored in the activation dtype
        for i, (a, b_) in enumerate(zip(got, want)):
            if a is None or not a.numel():
                continue
            rel = float((a.float() - b_.float()).norm() / (b_.float().norm() + 1e-12))
            assert rel < (out_tol if i < 2 else 1e-5), (i, rel)
        sums_got = torch.ops.rtseg.bn_bwd_sums(dense, x, ysave, mi, ss, 1, mask, d2)
        sums_want = torch.ops.rtseg.bn_bwd_sums(tot, x32, ysave32, mi, ss, 1, mask)
        torch.testing.assert_close(sums_got, sums_want, rtol=1e-5, atol=1e-4)


def _stdc_step(mod, x, sink_on, monkeypatch):
    monkeypatch.setattr(concat_mod, "_ENABLED", sink_on)
    m = copy.deepcopy(mod)
    xx = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(xx)
    torch.manual_seed(0)
    (y.float() * torch.randn(y.shape, device="cuda")).sum().backward()
    return y.detach().float(), xx.grad.float(), {k: p.grad.float() for k, p in m.named_parameters()}


@pytest.mark.parametrize("stride", [1, 2])
def test_stdc_module_sink_matches_torch_cat(stride, monkeypatch):
    from realtime_semantic_segmentation_pytorch_amd.models.stdc import STDCModule

    torch.manual_seed(1)
    mod = STDCModule(128, 256, stride, "relu").cuda().to(**CL).train()
    ops.convert_batchnorm(mod)
    x = torch.randn(4, 128, 32, 64, device="cuda").contiguous(**CL)
    y0, dx0, g0 = _stdc_step(mod, x, False, monkeypatch)
    y1, dx1, g1 = _stdc_step(mod, x, True, monkeypatch)
    torch.testing.assert_close(y1, y0, rtol=0, atol=0)  # the same kernels, stored twice
    rel = lambda a, b: float((a - b).norm() / (b.norm() + 1e-12))  # noqa: E731
    # backward: the slice is summed in fp32 inside the BN kernels instead of a bf16 add
    assert rel(dx1, dx0) < 2e-2, rel(dx1, dx0)
    for k in g0:
        assert rel(g1[k], g0[k]) < 3e-2, (k, rel(g1[k], g0[k]))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("act", ["relu", "none", "prelu"])
@pytest.mark.parametrize("train", [True, False])
def test_cat_bn_act_matches_cat_then_bn(dtype, act, train):
    """ops.cat_bn_act (per-part statistics, one finalize, per-part apply into the output slice,
    per-part backward on the gradient slice) vs bn_act of the materialised torch.cat: output,
    part gradients, BN parameter gradients and running statistics."""
    from realtime_semantic_segmentation_pytorch_amd.models.modules import Activation

    torch.manual_seed(0)
    widths = (32, 16, 24) if dtype == torch.bfloat16 else (12, 8, 4)
    c = sum(widths)
    bn = ops.convert_batchnorm(torch.nn.Sequential(torch.nn.BatchNorm2d(c))).cuda()[0]
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 2.0)
    bn.train(train)
    actm = Activation(act).cuda().to(dtype)  # (PReLU's weight in the activation dtype: no autocast here)
    parts0 = [(torch.randn(2, w, 9, 14, device="cuda") * (1 + i) + i).to(dtype).contiguous(
        memory_format=torch.channels_last) for i, w in enumerate(widths)]
    g = torch.randn(2, c, 9, 14, device="cuda")
    res = []
    for fused in (True, False):
        b = copy.deepcopy(bn)
        a = copy.deepcopy(actm)
        parts = [p.clone().requires_grad_(True) for p in parts0]
        before = concat_mod.CAT_BN_CALLS[0]
        if fused:
            y = ops.cat_bn_act(parts, b, a, act_module=a)
            assert concat_mod.CAT_BN_CALLS[0] == before + 1
        else:
            y = ops.bn_act(torch.cat(parts, dim=1), b, a, act_module=a)
        (y.float() * g).sum().backward()
        res.append((y.float().detach(), [p.grad.float() for p in parts], b.weight.grad.clone(), b.bias.grad.clone(),
                    b.running_mean.clone(), b.running_var.clone()))
    (y0, gp0, gw0, gb0, rm0, rv0), (y1, gp1, gw1, gb1, rm1, rv1) = res
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y0, y1, atol=tol, rtol=tol)
    for a_, b_ in zip(gp0, gp1):
        torch.testing.assert_close(a_, b_, atol=tol * b_.abs().max().item(), rtol=tol)
    torch.testing.assert_close(gw0, gw1, atol=tol * gw1.abs().max().item(), rtol=tol)
    torch.testing.assert_close(gb0, gb1, atol=tol * gb1.abs().max().item(), rtol=tol)
    torch.testing.assert_close(rm0, rm1, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rv0, rv1, atol=1e-5, rtol=1e-5)


def test_cgnet_block_uses_cat_bn():
    """CGNet's context-guided block runs its joint BN + PReLU through cat_bn_act on the GPU."""
    from realtime_semantic_segmentation_pytorch_amd.models.cgnet import CGBlock

    blk = ops.convert_batchnorm(CGBlock(64, 64, 1, 2)).cuda().to(memory_format=torch.channels_last).train()
    x = torch.randn(2, 64, 16, 24, device="cuda").contiguous(memory_format=torch.channels_last)
    before = concat_mod.CAT_BN_CALLS[0]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = blk(x)
    y.float().sum().backward()
    assert concat_mod.CAT_BN_CALLS[0] == before + 1


def _stem_step(mod, x, sink_on, monkeypatch, amp):
    monkeypatch.setattr(concat_mod, "_ENABLED", sink_on)
    m = copy.deepcopy(mod)
    xx = x.clone().requires_grad_(True)
    with torch.autocast(x.device.type, dtype=torch.bfloat16, enabled=amp):
        y = m(xx)
    gen = torch.Generator().manual_seed(0)
    (y.float() * torch.randn(y.shape, generator=gen).to(y.device)).sum().backward()
    return y, xx.grad.float(), {k: p.grad.float() for k, p in m.named_parameters()}


@pytest.mark.parametrize("amp", [False, True])
def test_bisenetv2_stem_concat_conv_without_cat(amp, monkeypatch):
    """K11 at a concat -> conv site (BiSeNetV2's stem, reference models/bisenetv2.py:84-96:
    ``conv_last(cat([left_branch(x), maxpool(x)]))``): the left BN stores into its slice of the
    concat buffer, the max pool runs inside the cat node into the other (pool2d_fwd_out) and
    its backward reads the gradient slice at its row stride.  No torch.cat runs; the result
    matches the same module on torch.cat and, in fp32, a CPU fp32 run of the stock module."""
    from realtime_semantic_segmentation_pytorch_amd.models.bisenetv2 import StemBlock

    torch.manual_seed(3)
    mod = StemBlock(3, 16).train()
    ref = copy.deepcopy(mod)
    mod = ops.convert_batchnorm(mod).cuda().to(**CL)
    x = torch.randn(2, 3, 64, 96)
    cats = []
    real_cat = torch.cat
    def spy(*a, **k):
        out = real_cat(*a, **k)
        if out.dim() == 4:  # the stem's concat (small 1-D cats of BN sums do not count)
            cats.append(tuple(out.shape))
        return out

    monkeypatch.setattr(torch, "cat", spy)
    y1, dx1, g1 = _stem_step(mod, x.cuda().contiguous(**CL), True, monkeypatch, amp)
    assert not cats, f"the sink path ran torch.cat: {cats}"
    monkeypatch.setattr(torch, "cat", real_cat)
    y0, dx0, g0 = _stem_step(mod, x.cuda().contiguous(**CL), False, monkeypatch, amp)
    rel = lambda a, b: float((a - b).norm() / (b.norm() + 1e-12))  # noqa: E731
    if amp:  # the BN slice gradient is summed in fp32 inside the kernel instead of a bf16 add
        assert rel(y1.float(), y0.float()) < 1e-2
        assert rel(dx1, dx0) < 2e-2, rel(dx1, dx0)
        for k in g0:
            assert rel(g1[k], g0[k]) < 3e-2, (k, rel(g1[k], g0[k]))
        return
    torch.testing.assert_close(y1, y0, rtol=1e-6, atol=1e-6)
    assert rel(dx1, dx0) < 1e-5, rel(dx1, dx0)
    yr, dxr, gr = _stem_step(ref.double(), x.double(), False, monkeypatch, False)
    assert rel(y1.double().cpu(), yr) < 1e-4
    assert rel(dx1.double().cpu(), dxr.double()) < 1e-4, rel(dx1.double().cpu(), dxr.double())
    for k in gr:
        assert rel(g1[k].double().cpu(), gr[k].double()) < 1e-3, (k, rel(g1[k].double().cpu(), gr[k].double()))


@pytest.mark.parametrize("act", ["relu", "prelu"])
@pytest.mark.parametrize("amp", [False, True])
def test_initial_block_pooled_sink(act, amp, monkeypatch):
    """The ENet-family InitialBlock (reference models/enet.py:38-48; 10 zoo networks):
    conv-BN-act || max-pool into one concat buffer.  ReLU: both parts are written in place;
    PReLU (unfused activation): the pool still runs into its slice, the conv part is copied.
    Against the same block on torch.cat (and, fp32, a CPU fp64 run)."""
    from realtime_semantic_segmentation_pytorch_amd.models.enet import InitialBlock

    torch.manual_seed(5)
    mod = InitialBlock(16, 64, act).train()
    ref = copy.deepcopy(mod)
    mod = ops.convert_batchnorm(mod).cuda().to(**CL)
    x = torch.randn(2, 16, 48, 80)
    y1, dx1, g1 = _stem_step(mod, x.cuda().contiguous(**CL), True, monkeypatch, amp)
    assert y1.dtype == (torch.bfloat16 if amp else torch.float32)
    y0, dx0, g0 = _stem_step(mod, x.cuda().contiguous(**CL), False, monkeypatch, amp)
    rel = lambda a, b: float((a - b).norm() / (b.norm() + 1e-12))  # noqa: E731
    if amp:
        assert rel(y1.float(), y0.float()) < 1e-2
        assert rel(dx1, dx0) < 2e-2, rel(dx1, dx0)
        for k in g0:
            assert rel(g1[k], g0[k]) < 3e-2, (k, rel(g1[k], g0[k]))
        return
    torch.testing.assert_close(y1, y0, rtol=1e-6, atol=1e-6)
    assert rel(dx1, dx0) < 1e-5, rel(dx1, dx0)
    yr, dxr, gr = _stem_step(ref.double(), x.double(), False, monkeypatch, False)
    assert rel(y1.double().cpu(), yr) < 1e-4
    assert rel(dx1.double().cpu(), dxr.double()) < 1e-4
    for k in gr:
        assert rel(g1[k].double().cpu(), gr[k].double()) < 1e-3, k
