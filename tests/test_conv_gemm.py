"""Pointwise (1 x 1, pad 0, stride 1 / 2) conv passes as plain GEMMs over channels-last pixel
rows (ops/conv.py gemm_fwd / gemm_dgrad / gemm_wgrad; hipBLASLt on the GPU) vs fp32 PyTorch
convolutions of the same bf16 operands: forward, data gradient with and without a residual
addend, fp32 weight gradient.  Reference layers: DDRNet's DAPPM 1 x 1s and the strided 1 x 1
projection shortcuts (reference models/ddrnet.py:168-219, :116-165).  The helpers run on the
CPU too, so the CPU suite checks the index algebra; the GPU cases check the routed autotune
candidate."""
import pytest
import torch
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd.ops import conv as conv_mod

CL = dict(memory_format=torch.channels_last)
# (n, cin, h, w, cout, stride) -- odd spatial sizes take the partial stride-2 rows / columns
GEOMS = [(2, 64, 9, 14, 32, 1), (3, 32, 11, 7, 64, 2), (1, 128, 16, 32, 256, 2), (4, 1024, 2, 4, 256, 1)]


def _devices():
    return ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _t(shape, g, dev, scale=1.0):
    return (torch.randn(shape, generator=g) * scale).to(dev, torch.bfloat16).contiguous(**CL)


def _close(got, ref, tol):
    torch.testing.assert_close(got.float(), ref, atol=tol * ref.abs().max().item() + 1e-6, rtol=tol)


@pytest.mark.parametrize("dev", _devices())
@pytest.mark.parametrize("geom", GEOMS)
def test_gemm_passes_match_conv(dev, geom):
    n, cin, h, w, cout, s = geom
    g = torch.Generator().manual_seed(0)
    x = _t((n, cin, h, w), g, dev)
    wt = (torch.randn(cout, cin, 1, 1, generator=g) * 0.1).to(dev, torch.bfloat16)
    wk = wt.permute(0, 2, 3, 1).contiguous()  # KRSC, as ops/conv.py weight_krsc
    y = conv_mod.gemm_fwd(x, wk, s)
    ref = F.conv2d(x.float(), wt.float(), None, s)
    assert y.shape == ref.shape and y.is_contiguous(**CL)
    _close(y, ref, 1e-2)

    dy = _t(ref.shape, g, dev)
    xr = x.float().requires_grad_(True)
    wr = wt.float().requires_grad_(True)
    F.conv2d(xr, wr, None, s).backward(dy.float())
    dx = conv_mod.gemm_dgrad(dy, wk, x.shape, s)
    assert dx.shape == x.shape and dx.is_contiguous(**CL)
    _close(dx, xr.grad, 1e-2)
    if s > 1:  # the rows / columns the stride skips get exactly zero
        mask = torch.ones_like(dx, dtype=torch.bool)
        mask[:, :, ::s, ::s] = False
        assert not dx[mask].any()
    addend = _t(x.shape, g, dev)
    dxa = conv_mod.gemm_dgrad(dy, wk, x.shape, s, addend)
    _close(dxa, xr.grad + addend.float(), 1e-2)
    dw = conv_mod.gemm_wgrad(x, dy, s)
    assert dw.shape == wt.shape and dw.dtype == torch.float32
    _close(dw, wr.grad, 1e-3 if dev == "cuda" else 1e-2)


def test_gemm_ok_geometries():
    ok = conv_mod.gemm_ok
    assert ok(torch.nn.Conv2d(64, 128, 1, 2, bias=False))
    assert ok(torch.nn.Conv2d(1024, 256, 1, bias=False))
    assert not ok(torch.nn.Conv2d(64, 128, 1, 2, padding=1, bias=False))
    assert not ok(torch.nn.Conv2d(64, 128, 3, 1, 1, bias=False))
    assert not ok(torch.nn.Conv2d(64, 128, 1, 4, bias=False))
    assert not ok(torch.nn.Conv2d(64, 128, 1, groups=2, bias=False))


@pytest.mark.gpu
@pytest.mark.parametrize("block", ["RB", "RBB"])
def test_gemm_routed_downsample_block(monkeypatch, block):
    """A downsampling DDRNet block (3 x 3 stride-2 conv + strided 1 x 1 projection) with the
    GEMM candidate forced for the 1 x 1 passes vs the autotuned path without it: each one's
    forward, input and parameter gradients against an fp32 CPU run of the same block, the GEMM
    path within 1.5 x the other's error (+ a bf16-rounding floor), and the 1 x 1 passes really
    took the GEMM path."""
    import copy

    from realtime_semantic_segmentation_pytorch_amd import ops
    from realtime_semantic_segmentation_pytorch_amd.models import ddrnet

    assert ops.load(), "HIP extension must load on the GPU box"
    torch.manual_seed(0)
    net = ops.convert_batchnorm(getattr(ddrnet, block)(64, 128, 2)).cuda().to(**CL).train()
    x0 = torch.randn(2, 64, 32, 96, device="cuda").contiguous(**CL)
    gy = torch.randn(2, 128, 16, 48, device="cuda")
    res, calls = [], []
    monkeypatch.setattr(conv_mod, "_PHASE_FUSE", False)  # the shortcut dgrad as its own (GEMM) pass
    for name in ("gemm_fwd", "gemm_dgrad", "gemm_wgrad"):
        def spy(*a, _f=getattr(conv_mod, name), _n=name, **k):
            calls[-1].add(_n)
            return _f(*a, **k)

        monkeypatch.setattr(conv_mod, name, spy)
    for mode in ("1", "0"):
        monkeypatch.setenv("RTSEG_CONV_GEMM", mode)
        if mode == "1":  # the first candidate everywhere, no timing
            monkeypatch.setenv("RTSEG_CONV_MFMA", "1")
        else:
            monkeypatch.delenv("RTSEG_CONV_MFMA", raising=False)
        calls.append(set())
        net.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = net(x)
        (y.float() * gy).sum().backward()
        res.append((y.float().detach(), x.grad.float().clone(),
                    {n: p.grad.float().clone() for n, p in net.named_parameters()}))
    ref = copy.deepcopy(net).cpu().float()
    ref.zero_grad(set_to_none=True)
    xr = x0.cpu().clone().requires_grad_(True)
    yr = ref(xr)
    (yr * gy.cpu()).sum().backward()
    gpr = {n: p.grad for n, p in ref.named_parameters()}
    (y0, gx0, gp0), (y1, gx1, gp1) = res

    def rel(a, b):
        return ((a.cpu() - b).norm() / b.norm().clamp_min(1e-12)).item()

    def ok(e_gemm, e_other, floor):
        return e_gemm <= max(1.5 * e_other, floor)

    assert ok(rel(y0, yr), rel(y1, yr), 1e-2), (rel(y0, yr), rel(y1, yr))
    assert ok(rel(gx0, xr.grad), rel(gx1, xr.grad), 2e-2), (rel(gx0, xr.grad), rel(gx1, xr.grad))
    for n, g in gpr.items():
        assert ok(rel(gp0[n], g), rel(gp1[n], g), 2e-2), (n, rel(gp0[n], g), rel(gp1[n], g))
    assert calls[0] == {"gemm_fwd", "gemm_dgrad", "gemm_wgrad"}, calls[0]
    assert not calls[1], calls[1]


def test_masked_addend_materialize_cpu():
    """MaskedAddend (ops/conv.py): the channels-last bit order of the BN activation mask."""
    g = torch.randn(2, 16, 3, 5).to(torch.bfloat16).contiguous(**CL)
    m = torch.rand(2, 16, 3, 5) > 0.5
    flat = m.permute(0, 2, 3, 1).reshape(-1, 8).to(torch.uint8)  # element e -> byte e // 8, bit e % 8
    bits = (flat << torch.arange(8, dtype=torch.uint8)).sum(1).to(torch.uint8)
    out = conv_mod.MaskedAddend(g, bits).materialize()
    assert torch.equal(out, g * m.to(g.dtype))


@pytest.mark.gpu
@pytest.mark.parametrize("block", ["RB"])  # RBB's twin is two 1 x 1s (stride 1 and 2): not fused
def test_twin_phase_fused_shortcut_dgrad(monkeypatch, block):
    """A downsampling block's strided 1 x 1 shortcut dgrad as a GEMM added by the 3 x 3 dgrad's
    phase-(0, 0) launch (ops/conv.py _TwinConvFn, RTSEG_TWIN_PHASE) vs the separate pass: each
    against an fp32 CPU run of the block, the fused path within 1.5 x the other's error (+ a
    bf16 floor), and the fused path really ran."""
    import copy

    from realtime_semantic_segmentation_pytorch_amd import ops
    from realtime_semantic_segmentation_pytorch_amd.models import ddrnet

    assert ops.load(), "HIP extension must load on the GPU box"
    monkeypatch.setenv("RTSEG_TWIN_CONV", "1")
    torch.manual_seed(0)
    net = ops.convert_batchnorm(getattr(ddrnet, block)(64, 128, 2)).cuda().to(**CL).train()
    x0 = torch.randn(2, 64, 34, 98, device="cuda").contiguous(**CL)
    gy = torch.randn(2, 128, 17, 49, device="cuda")
    res = []
    for on in (True, False):
        monkeypatch.setattr(conv_mod, "_PHASE_FUSE", on)
        before = conv_mod.PHASE_FUSED[0]
        net.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = net(x)
        (y.float() * gy).sum().backward()
        assert (conv_mod.PHASE_FUSED[0] > before) == on
        res.append((y.float().detach(), x.grad.float().clone(),
                    {n: p.grad.float().clone() for n, p in net.named_parameters()}))
    ref = copy.deepcopy(net).cpu().float()
    ref.zero_grad(set_to_none=True)
    xr = x0.cpu().clone().requires_grad_(True)
    (ref(xr) * gy.cpu()).sum().backward()
    (_, gx0, gp0), (_, gx1, gp1) = res

    def rel(a, b):
        return ((a.cpu() - b).norm() / b.norm().clamp_min(1e-12)).item()

    assert rel(gx0, xr.grad) <= max(1.5 * rel(gx1, xr.grad), 2e-2), (rel(gx0, xr.grad), rel(gx1, xr.grad))
    for n, p in ref.named_parameters():
        assert rel(gp0[n], p.grad) <= max(1.5 * rel(gp1[n], p.grad), 2e-2), n
