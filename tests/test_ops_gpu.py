"""Numerics of the HIP kernels vs plain-PyTorch fp32 references (run on MI355X)."""
import math

import pytest
import torch
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lib_loaded():
    assert ops.load(), "HIP extension must load on the GPU box"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [False, True])
@pytest.mark.parametrize("align", [True, False])
@pytest.mark.parametrize("shape,size", [((2, 16, 7, 9), (28, 36)), ((1, 24, 16, 32), (128, 256)),
                                        ((2, 8, 32, 64), (16, 32)), ((1, 16, 1, 1), (16, 32)),
                                        # odd channel counts: dense channels-last output staged
                                        # through LDS (19-class logits, RGB)
                                        ((2, 19, 16, 24), (64, 96)), ((1, 3, 9, 11), (40, 50))])
def test_interp_fwd_bwd(dtype, cl, align, shape, size):
    _lib_loaded()
    torch.manual_seed(0)
    x = torch.randn(shape, device=DEV, dtype=dtype)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = ops.interpolate(x, size, align)
    xr = x.detach().float().requires_grad_(True)
    yr = F.interpolate(xr, size, mode="bilinear", align_corners=align)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    gtol = 1e-4 if dtype == torch.float32 else 5e-2
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=gtol * max(1.0, xr.grad.abs().max().item()), rtol=gtol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,size", [((1, 19, 128, 256), (1024, 2048)), ((2, 19, 9, 13), (72, 104)),
                                        ((1, 3, 20, 24), (80, 96))])
@pytest.mark.parametrize("align", [True, False])
def test_interp_final_upsample_rows(monkeypatch, dtype, shape, size, align):
    """The row-staged kernel (interp_fwd_cl_rows: a dense channels-last few-channel output,
    >= x4 wide -- the models' final logits upsample in inference) against fp32 PyTorch and
    against the per-pixel kernel it replaces (RTSEG_INTERP_ROWS=0 in a subprocess is not needed:
    the two differ only by the fp32 blend order, <= 1 bf16 ulp)."""
    _lib_loaded()
    torch.manual_seed(4)
    x = torch.randn(shape, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y = ops.interpolate(x, size, align)
    ref = F.interpolate(x.float(), size, mode="bilinear", align_corners=align)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    if dtype == torch.float32:
        torch.testing.assert_close(y, ref, atol=1e-5, rtol=1e-5)
    else:
        torch.testing.assert_close(y.float(), ref, rtol=2.0 ** -8, atol=1e-3 * ref.abs().max().item())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", [None, "relu"])
def test_interp_skip_act(dtype, act):
    _lib_loaded()
    torch.manual_seed(1)
    x = torch.randn(2, 32, 16, 32, device=DEV, dtype=dtype).contiguous(memory_format=torch.channels_last)
    s = torch.randn(2, 32, 64, 128, device=DEV, dtype=dtype).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    s.requires_grad_(True)
    y = ops.interpolate(x, (64, 128), True, skip=s, act=act)
    xr = x.detach().float().requires_grad_(True)
    sr = s.detach().float().requires_grad_(True)
    yr = F.interpolate(xr, (64, 128), mode="bilinear", align_corners=True) + sr
    if act == "relu":
        # relu mask taken from the kernel output: in bf16 a pre-activation within
        # rounding of 0 may legitimately land on either side
        yr = yr * (y.detach() > 0).float()
    tol = 1e-5 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    gtol = 1e-4 if dtype == torch.float32 else 6e-2
    torch.testing.assert_close(s.grad.float(), sr.grad, atol=gtol, rtol=gtol)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=gtol * xr.grad.abs().max().item(), rtol=gtol)


def _labels(n, h, w, c, ignore_frac=0.1, seed=0):
    g = torch.Generator().manual_seed(seed)
    lab = torch.randint(0, c, (n, h, w), generator=g)
    lab[torch.rand((n, h, w), generator=g) < ignore_frac] = 255
    return lab.to(DEV)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("scale_logits", [0.1, 3.0])  # small logits -> top-k branch; large -> threshold
@pytest.mark.parametrize("hw,lhw", [((16, 32), (128, 256)), ((32, 64), (32, 64)), ((9, 13), (70, 100)),
                                    ((64, 128), (128, 256)), ((32, 64), (128, 256)), ((37, 51), (70, 100))])
def test_ohem_loss_fused(dtype, scale_logits, hw, lhw):
    _lib_loaded()
    torch.manual_seed(2)
    n, c = 2, 19
    logits = (torch.randn(n, c, *hw, device=DEV) * scale_logits).to(dtype)
    logits = logits.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    labels = _labels(n, *lhw, c)
    loss = ops.seg_cross_entropy(logits, labels, mode=ops.MODE_OHEM, ohem_thrs=0.7)
    lr_ = logits.detach().float().requires_grad_(True)
    ref = ops.seg_cross_entropy_reference(lr_, labels.cpu().to(DEV), mode=ops.MODE_OHEM, ohem_thrs=0.7)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(loss, ref, atol=tol, rtol=tol)
    loss.backward()
    ref.backward()
    gmax = lr_.grad.abs().max().item()
    torch.testing.assert_close(logits.grad.float(), lr_.grad, atol=max(1e-7, 2e-2 * gmax), rtol=5e-2)


@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("mode", [1, 2])
def test_ce_loss_modes(weighted, mode):
    _lib_loaded()
    torch.manual_seed(3)
    n, c = 2, 19
    logits = torch.randn(n, c, 16, 32, device=DEV, requires_grad=True)
    labels = _labels(n, 128, 256, c, seed=4)
    w = torch.rand(c, device=DEV) + 0.5 if weighted else None
    loss = ops.seg_cross_entropy(logits, labels, mode=mode, class_weight=w)
    lr_ = logits.detach().clone().requires_grad_(True)
    ref = ops.seg_cross_entropy_reference(lr_, labels, mode=mode, class_weight=w)
    torch.testing.assert_close(loss, ref, atol=1e-4, rtol=1e-4)
    loss.backward()
    ref.backward()
    torch.testing.assert_close(logits.grad, lr_.grad, atol=1e-6 + 1e-3 * lr_.grad.abs().max().item(), rtol=1e-3)


@pytest.mark.parametrize("c,hw,lhw,cl", [(40, (12, 20), (96, 160), True), (40, (24, 40), (24, 40), False),
                                         (19, (16, 32), (128, 256), False), (7, (5, 300), (40, 2400), True),
                                         (150, (16, 16), (64, 64), True)])
@pytest.mark.parametrize("u8", [False, True])
def test_loss_class_counts_layouts(c, hw, lhw, cl, u8):
    _lib_loaded()
    torch.manual_seed(7)
    logits = torch.randn(2, c, *hw, device=DEV) * 2
    if cl:
        logits = logits.contiguous(memory_format=torch.channels_last)
    logits.requires_grad_(True)
    labels = _labels(2, *lhw, c, seed=8)
    loss = ops.seg_cross_entropy(logits, labels.to(torch.uint8) if u8 else labels)
    lr_ = logits.detach().clone().requires_grad_(True)
    ref = ops.seg_cross_entropy_reference(lr_, labels)
    torch.testing.assert_close(loss, ref, atol=1e-4, rtol=1e-4)
    loss.backward()
    ref.backward()
    torch.testing.assert_close(logits.grad, lr_.grad, atol=1e-6 + 1e-3 * lr_.grad.abs().max().item(), rtol=1e-3)


def test_aux_loss_nearest_labels():
    _lib_loaded()
    torch.manual_seed(5)
    logits = torch.randn(2, 19, 16, 32, device=DEV, requires_grad=True)
    labels = _labels(2, 128, 256, 19, seed=6)
    loss = ops.seg_cross_entropy(logits, labels, resize_logits=False)
    lr_ = logits.detach().clone().requires_grad_(True)
    ref = ops.seg_cross_entropy_reference(lr_, labels, resize_logits=False)
    torch.testing.assert_close(loss, ref, atol=1e-4, rtol=1e-4)
    loss.backward()
    ref.backward()
    torch.testing.assert_close(logits.grad, lr_.grad, atol=1e-6 + 1e-3 * lr_.grad.abs().max().item(), rtol=1e-3)


def test_loss_no_host_sync():
    """The fused loss must not synchronise with the host (graph-capturable)."""
    _lib_loaded()
    logits = torch.randn(2, 19, 16, 32, device=DEV, requires_grad=True)
    labels = _labels(2, 128, 256, 19)
    torch.cuda.set_sync_debug_mode("error")
    try:
        loss = ops.seg_cross_entropy(logits, labels)
        loss.backward()
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert math.isfinite(float(loss))


@pytest.mark.parametrize("form", ["0", "1", "2"])
@pytest.mark.parametrize("scale", [2.0, 200.0])  # 200: a run's lse spans > 2^60 -> per-pixel shift
@pytest.mark.parametrize("align", [True, False])
def test_loss_bwd_run_forms(monkeypatch, form, scale, align):
    """The x8 upsampled 19-class backward: round-4 tile form (0), first run form (1) and the packed
    run form with the exp2 shift and LDS one-hot terms (2, default) against the fp32 reference."""
    _lib_loaded()
    monkeypatch.setenv("RTSEG_LOSS_BWD_RUN", form)
    torch.manual_seed(11)
    logits = (torch.randn(2, 19, 24, 40, device=DEV) * scale).contiguous(memory_format=torch.channels_last)
    logits.requires_grad_(True)
    labels = _labels(2, 192, 320, 19, seed=12)
    for mode in (ops.MODE_OHEM, 1):
        logits.grad = None
        loss = ops.seg_cross_entropy(logits, labels.to(torch.uint8), mode=mode, align_corners=align)
        lr_ = logits.detach().clone().requires_grad_(True)
        ref = ops.seg_cross_entropy_reference(lr_, labels, mode=mode, align_corners=align)
        torch.testing.assert_close(loss, ref, atol=1e-4, rtol=1e-4)
        loss.backward()
        ref.backward()
        assert torch.isfinite(logits.grad).all()
        torch.testing.assert_close(logits.grad, lr_.grad, atol=1e-6 + 1e-3 * lr_.grad.abs().max().item(),
                                   rtol=1e-3)
