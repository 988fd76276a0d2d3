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
