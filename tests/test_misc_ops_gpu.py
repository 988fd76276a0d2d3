"""KD KL loss, confusion matrix and fused optimizer+EMA HIP kernels vs PyTorch fp32 references."""
import copy

import pytest
import torch
import torch.nn as nn

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.ops.optim import FusedAdam, FusedAdamW, FusedSGD

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _lib():
    assert ops.load(), "HIP extension must load on the GPU box"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [False, True])
@pytest.mark.parametrize("shape,temp", [((2, 19, 32, 64), 4.0), ((1, 7, 9, 13), 1.0), ((3, 40, 5, 6), 2.5)])
def test_kd_kl_fwd_bwd(dtype, cl, shape, temp):
    torch.manual_seed(0)
    s = (torch.randn(shape, device=DEV) * 3).to(dtype)
    t = (torch.randn(shape, device=DEV) * 3).to(dtype)
    if cl:
        s = s.contiguous(memory_format=torch.channels_last)
        t = t.contiguous(memory_format=torch.channels_last)
    s.requires_grad_(True)
    loss = ops.kd_kl_div(s, t, temp)
    sr = s.detach().float().requires_grad_(True)
    ref = ops.kd_kl_div_reference(sr, t.float(), temp)
    torch.testing.assert_close(loss.float(), ref, rtol=1e-4, atol=1e-6)
    loss.backward(torch.tensor(0.7, device=DEV))
    ref.backward(torch.tensor(0.7, device=DEV))
    scale = sr.grad.abs().max().item()
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(s.grad.float(), sr.grad, atol=tol * scale, rtol=tol)
    if cl:
        assert s.grad.is_contiguous(memory_format=torch.channels_last)


def test_kd_no_host_sync():
    s = torch.randn(2, 19, 16, 32, device=DEV, requires_grad=True)
    t = torch.randn(2, 19, 16, 32, device=DEV)
    torch.cuda.set_sync_debug_mode("error")
    try:
        loss = ops.kd_kl_div(s, t, 4.0)
        loss.backward()
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert torch.isfinite(loss).item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [False, True])
@pytest.mark.parametrize("c", [19, 3, 150])
def test_confmat(dtype, cl, c):
    torch.manual_seed(1)
    x = torch.randn(2, c, 33, 47, device=DEV).to(dtype)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, c, (2, 33, 47), device=DEV)
    y[:, ::5] = 255
    cm = ops.confusion_matrix(x, y, c, 255)
    ref = ops.confusion_matrix_reference(x.float().cpu(), y.cpu(), c, 255)
    assert cm.dtype == torch.int64
    torch.testing.assert_close(cm.cpu(), ref)


def _model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Conv2d(3, 16, 3, bias=False), nn.BatchNorm2d(16), nn.ReLU(),
                         nn.Conv2d(16, 40000 // 16, 1), nn.Flatten(), nn.Linear(2500 * 4, 3)).to(DEV)


@pytest.mark.parametrize("cl", [False, True])
@pytest.mark.parametrize("kind", ["sgd", "sgd_nesterov", "adam", "adamw"])
def test_fused_optimizer_matches_torch(kind, cl):
    m_ref = _model()
    if cl:  # channels-last conv weights: dense but not contiguous -- the fused kernel must take them
        m_ref = m_ref.to(memory_format=torch.channels_last)
    m_fus = copy.deepcopy(m_ref)
    ema = copy.deepcopy(m_fus)
    ema_ref = copy.deepcopy(m_ref)
    if kind.startswith("sgd"):
        kw = dict(lr=0.05, momentum=0.9, weight_decay=1e-4, nesterov=kind == "sgd_nesterov")
        o_ref, o_fus = torch.optim.SGD(m_ref.parameters(), **kw), FusedSGD(m_fus.parameters(), **kw)
    elif kind == "adam":
        o_ref, o_fus = torch.optim.Adam(m_ref.parameters(), lr=1e-3), FusedAdam(m_fus.parameters(), lr=1e-3)
    else:
        kw = dict(lr=1e-3, weight_decay=0.01)
        o_ref, o_fus = torch.optim.AdamW(m_ref.parameters(), **kw), FusedAdamW(m_fus.parameters(), **kw)
    pairs = [(p, e.data) for p, e in zip(m_fus.parameters(), ema.parameters())]
    o_fus.attach_ema(pairs)
    x = torch.randn(4, 3, 4, 4, device=DEV)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    for it in range(1, 5):
        for m, o in ((m_ref, o_ref), (m_fus, o_fus)):
            o.zero_grad()
            m(x).square().mean().backward()
        decay = it / 10
        o_fus.ema_weight = 1.0 - decay
        o_ref.step()
        o_fus.step()
        assert o_fus.last_step_fused
        with torch.no_grad():
            for e, p in zip(ema_ref.parameters(), m_ref.parameters()):
                e.lerp_(p, 1.0 - decay)
    for a, b in zip(m_ref.parameters(), m_fus.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    for a, b in zip(ema_ref.parameters(), ema.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    # state layout is torch's: a torch optimizer can resume from the fused one's state dict
    sd = o_fus.state_dict()
    o2 = type(o_ref)(m_fus.parameters(), lr=1e-3)
    o2.load_state_dict(sd)


def test_ema_lerp_buffers():
    from realtime_semantic_segmentation_pytorch_amd.ops.optim import ema_lerp_

    src = [torch.randn(n, device=DEV) for n in (5, 70000, 1)]
    ema = [torch.randn_like(s) for s in src]
    ref = [e.clone().lerp_(s, 0.3) for e, s in zip(ema, src)]
    ema_lerp_(list(zip(src, ema)), 0.3)
    for a, b in zip(ema, ref):
        torch.testing.assert_close(a, b)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [False, True])
def test_colorize_matches_reference(dtype, cl):
    torch.manual_seed(7)
    x = torch.randn(2, 19, 33, 50, device=DEV).to(dtype)
    x[:, 3] = x[:, 5]  # ties -> first maximum
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    cmap = torch.randint(0, 256, (19, 3), dtype=torch.uint8, device=DEV)
    img = torch.randint(0, 256, (2, 33, 50, 3), dtype=torch.uint8, device=DEV)
    cls, rgb, blend = ops.colorize(x, cmap, img, 0.3)
    rc, rr, rb = ops.colorize_reference(x.float().cpu(), cmap.cpu(), img.cpu(), 0.3)
    assert torch.equal(cls.cpu(), rc) and torch.equal(rgb.cpu(), rr) and torch.equal(blend.cpu(), rb)
    cls2, _, none = ops.colorize(x, cmap)
    assert none is None and torch.equal(cls2, cls)


@pytest.mark.parametrize("axis,d,dt,cin,cout", [(0, 2, torch.float32, 8, 8), (1, 16, torch.float32, 4, 16),
                                                (0, 8, torch.bfloat16, 16, 4), (1, 4, torch.bfloat16, 8, 8)])
def test_tap_conv_gpu_vs_cpu_fp64(axis, d, dt, cin, cout):
    """TapConv2d (CFPNet's narrow dilated 1-D convs, ops/tapconv.py) on the GPU vs a CPU fp64
    F.conv2d -- the GPU reference would be the MIOpen path this module avoids."""
    import torch.nn.functional as F

    torch.manual_seed(0)
    ks, pad, dil = ((3, 1), (d, 0), (d, 1)) if axis == 0 else ((1, 3), (0, d), (1, d))
    conv = nn.Conv2d(cin, cout, ks, padding=pad, dilation=dil, bias=False)
    assert ops.tapconv_ok(conv)
    x = torch.randn(2, cin, 64, 128).contiguous(memory_format=torch.channels_last)
    g = torch.randn(2, cout, 64, 128)
    xr = x.double().requires_grad_(True)
    wr = conv.weight.detach().double().requires_grad_(True)
    ref = F.conv2d(xr, wr, None, 1, pad, dil)
    gxr, gwr = torch.autograd.grad(ref, (xr, wr), g.double())
    m = copy.deepcopy(conv).cuda()
    m.__class__ = ops.TapConv2d
    xc = x.cuda().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dt == torch.bfloat16):
        out = m(xc)
    gx, gw = torch.autograd.grad(out, (xc, m.weight), g.cuda().to(out.dtype))
    tol = dict(atol=5e-2, rtol=5e-2) if dt == torch.bfloat16 else dict(atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(out.float().cpu(), ref.float(), **tol)
    torch.testing.assert_close(gx.float().cpu(), gxr.float(), **tol)
    torch.testing.assert_close(gw.float().cpu(), gwr.float(), **dict(tol, atol=tol["atol"] * 20))


@pytest.mark.no_guard
@pytest.mark.parametrize("key", ["cgnet", "dabnet", "ddrnet"])
def test_inference_engine_bf16_matches_eager_autocast(key):
    """utils/inference.py: the graph engine (weights pre-cast to bf16 on a private copy) gives
    the eager bf16-autocast output of the same model, and leaves the caller's model fp32."""
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.models import get_model
    from realtime_semantic_segmentation_pytorch_amd.utils.inference import InferenceEngine

    c = BaseConfig()
    c.model, c.num_class = key, 19
    torch.manual_seed(0)
    m = get_model(c).cuda().eval().to(memory_format=torch.channels_last)
    x = torch.randn(1, 3, 128, 256, device="cuda")
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        ref = ops.materialize(m(x.contiguous(memory_format=torch.channels_last))).float()
    eng = InferenceEngine(m, (1, 3, 128, 256), dtype=torch.bfloat16)
    out = eng(x).float()
    assert all(p.dtype == torch.float32 for p in m.parameters())
    assert torch.isfinite(out).all()
    err = (out - ref).abs().max().item()
    assert err <= 0.05 * ref.abs().max().item() + 1e-2, err


@pytest.mark.no_guard
@pytest.mark.parametrize("key", ["dfanet", "espnet", "icnet"])
def test_inference_engine_bf16_input_bounded(key):
    """The engine's bf16 static input (utils/inference.py) rounds the image before the model; on the
    models whose image-side ops (input pyramids, pooled / resized image shortcuts) run in fp32 under
    eager autocast, the engine's distance to the fp32 eval output stays within 1.5x eager
    autocast's own distance (+ a small floor), and ``input_dtype=torch.float32`` is as close as
    eager autocast."""
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.models import get_model
    from realtime_semantic_segmentation_pytorch_amd.utils.inference import InferenceEngine

    c = BaseConfig()
    c.model, c.num_class = key, 19
    torch.manual_seed(0)
    m = get_model(c).cuda().eval().to(memory_format=torch.channels_last)
    x = torch.randn(1, 3, 256, 512, device="cuda")
    xc = x.contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        ref = ops.materialize(m(xc)).float()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            eager = ops.materialize(m(xc)).float()
    rel = lambda a: ((a - ref).norm() / ref.norm()).item()  # noqa: E731
    e_eager = rel(eager)
    e_bf16_in = rel(InferenceEngine(m, (1, 3, 256, 512), dtype=torch.bfloat16)(x).float())
    e_fp32_in = rel(InferenceEngine(m, (1, 3, 256, 512), dtype=torch.bfloat16, input_dtype=torch.float32)(x).float())
    assert e_bf16_in <= 1.5 * e_eager + 2e-3, (e_bf16_in, e_eager)
    assert e_fp32_in <= 1.5 * e_eager + 1e-3, (e_fp32_in, e_eager)
