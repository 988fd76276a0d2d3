"""Weights-resident halo conv (csrc/kernels/conv_wres.hip) and halo-tiled weight gradient
(csrc/kernels/conv_whalo.hip) vs fp32 PyTorch: forward (+ BN-statistics
slab) of 3x3 / stride-1 / pad-1 convs with Cin = 64 and the data gradient (+ residual-gradient
addend) of such convs with Cout = 64 -- partial tiles (H % 8, W % 32), several 64-channel output
slices, fewer tiles than blocks, and many tiles per block (statistics summed over a block's tiles
before its slab row).  Reference layers: DDRNet-23 layer1 RB blocks (ddrnet.py:168-191)."""
import pytest
import torch
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd import ops
from _tol import bf16_close, f32_close  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _mask_bits(shape, seed):
    """Random activation bit mask of a channels-last bf16 tensor (ops/bn.py kMaskBits layout)."""
    g = torch.Generator().manual_seed(seed)
    n = shape[0] * shape[1] * shape[2] * shape[3] // 8
    return torch.randint(0, 256, (n,), generator=g, dtype=torch.uint8).to(DEV)


def _addend_ref(add, bits, mode):
    """What the dgrad epilogue adds: nothing, the addend, or the addend where its mask bit is set
    (element e of the channels-last order in bit e % 8 of byte e / 8)."""
    if not mode:
        return 0.0
    a = add.float()
    if mode != "masked":
        return a
    n, c, h, w = add.shape
    m = torch.stack([(bits >> i) & 1 for i in range(8)], dim=1).reshape(n, h, w, c).permute(0, 3, 1, 2)
    return a * m.float()

# forward geometries (n, h, w, cout), Cin = 64
FWD = [(2, 17, 70, 64), (3, 8, 64, 128), (1, 5, 7, 64), (8, 130, 256, 64), (2, 33, 97, 192)]
# data-gradient geometries (n, h, w, cin) of forward convs with Cout = 64
DGRAD = [(2, 17, 70, 64), (3, 9, 40, 128), (8, 66, 256, 64), (1, 6, 33, 192)]


@pytest.fixture(autouse=True)
def _lib():
    assert ops.load(), "HIP extension must load on the GPU box"


def _t(shape, g, scale=1.0):
    return (torch.randn(shape, generator=g) * scale).to(DEV, torch.bfloat16)


def _close(got, ref, tol):
    torch.testing.assert_close(got.float(), ref, atol=tol * ref.abs().max().item() + 1e-6, rtol=tol)


@pytest.mark.parametrize("geom", FWD)
def test_wres_forward_and_stats(geom):
    n, h, w, cout = geom
    g = torch.Generator().manual_seed(0)
    x = _t((n, 64, h, w), g).contiguous(memory_format=torch.channels_last)
    wt = _t((cout, 64, 3, 3), g, 1 / 24)
    wk = wt.permute(0, 2, 3, 1).contiguous()
    y, part = torch.ops.rtseg.conv_wres(x, wk, [1, 1], [1, 1], [1, 1], True)
    ref = F.conv2d(x.float(), wt.float(), None, 1, 1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    bf16_close(y, ref)
    rf = ref.double()  # the slab holds the statistics of the fp32 outputs (the accumulators)
    torch.testing.assert_close(part[:, :cout].double().sum(0), rf.sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[:, cout:].double().sum(0), rf.square().sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    assert part.shape[0] <= 256
    y1, p1 = torch.ops.rtseg.conv_wres(x, wk, [1, 1], [1, 1], [1, 1], True)
    assert torch.equal(p1, part) and torch.equal(y1, y)  # deterministic
    y2, p2 = torch.ops.rtseg.conv_wres(x, wk, [1, 1], [1, 1], [1, 1], False)
    assert torch.equal(y2, y) and (p2 is None or p2.numel() == 0)


@pytest.mark.parametrize("geom", FWD)
@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("with_res", [False, True])
def test_wres_inference_bn_epilogue(geom, act, with_res):
    """conv_wres_eval: act(conv * scale + shift (+ residual)) from the fp32 accumulators (batch-1
    inference of the 64-channel 3 x 3 layers) against fp32; the conv part is the training
    kernel's (same accumulation): equal to applying the epilogue to its fp32 outputs."""
    n, h, w, cout = geom
    g = torch.Generator().manual_seed(5)
    x = _t((n, 64, h, w), g).contiguous(memory_format=torch.channels_last)
    wt = _t((cout, 64, 3, 3), g, 1 / 24)
    wk = wt.permute(0, 2, 3, 1).contiguous()
    ss = torch.cat([torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g)]).to(DEV).contiguous()
    res = _t((n, cout, h, w), g).contiguous(memory_format=torch.channels_last) if with_res else None
    y = torch.ops.rtseg.conv_wres_eval(x, wk, [1, 1], [1, 1], [1, 1], ss, res, act)
    ref = F.conv2d(x.float(), wt.float(), None, 1, 1) * ss[:cout].view(1, -1, 1, 1) + ss[cout:].view(1, -1, 1, 1)
    if with_res:
        ref = ref + res.float()
    ref = ref.relu() if act == 1 else ref.clamp(0, 6) if act == 2 else ref
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    bf16_close(y, ref)
    assert torch.equal(y, torch.ops.rtseg.conv_wres_eval(x, wk, [1, 1], [1, 1], [1, 1], ss, res, act))


@pytest.mark.parametrize("geom", DGRAD)
@pytest.mark.parametrize("with_addend", [False, True, "masked"])
def test_wres_dgrad(geom, with_addend):
    n, h, w, cin = geom
    g = torch.Generator().manual_seed(2)
    cl = dict(memory_format=torch.channels_last)
    wt = _t((64, cin, 3, 3), g, 1 / 24)
    dy = _t((n, 64, h, w), g).contiguous(**cl)
    add = _t((n, cin, h, w), g).contiguous(**cl)
    bits = _mask_bits(add.shape, 3)
    dx = torch.ops.rtseg.conv_wres_dgrad(dy, wt.permute(1, 2, 3, 0).contiguous(), [n, cin, h, w], [1, 1], [1, 1],
                                         [1, 1], add if with_addend else None, bits if with_addend == "masked" else None)
    ref = torch.nn.grad.conv2d_input((n, cin, h, w), wt.float(), dy.float(), 1, 1, 1)
    bf16_close(dx, ref + _addend_ref(add, bits, with_addend))


def test_wres_rejects_other_shapes():
    g = torch.Generator().manual_seed(1)
    x = _t((1, 128, 8, 32), g).contiguous(memory_format=torch.channels_last)
    wk = _t((64, 3, 3, 128), g)
    with pytest.raises(RuntimeError, match="conv_wres"):
        torch.ops.rtseg.conv_wres(x, wk, [1, 1], [1, 1], [1, 1], False)
    x = _t((1, 64, 8, 32), g).contiguous(memory_format=torch.channels_last)
    with pytest.raises(RuntimeError, match="conv_wres"):  # stride 2
        torch.ops.rtseg.conv_wres(x, _t((64, 3, 3, 64), g), [2, 2], [1, 1], [1, 1], False)


def test_wres_routed_training_step(monkeypatch):
    """DDRNet RB chain (64 channels) with conv_wres forced first vs the gather kernel: outputs and
    gradients agree up to bf16 rounding, and the routing really called the new kernels."""
    from realtime_semantic_segmentation_pytorch_amd.models.ddrnet import RB
    from realtime_semantic_segmentation_pytorch_amd.ops import conv as conv_mod

    torch.manual_seed(0)
    net = ops.convert_batchnorm(torch.nn.Sequential(RB(64, 64), RB(64, 64))).to(DEV)
    net = net.to(memory_format=torch.channels_last).train()
    x0 = torch.randn(2, 64, 24, 72, device=DEV).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(2, 64, 24, 72, device=DEV)
    calls = []

    class _Spy:  # records which rtseg ops the conv routing calls
        def __getattr__(self, name):
            calls[-1].add(name)
            return getattr(torch.ops.rtseg, name)

    spy = _Spy()
    monkeypatch.setattr(conv_mod, "ops", lambda: spy)
    res = []
    for env in ({"RTSEG_CONV_MFMA": "1", "RTSEG_CONV_WRES": "1"}, {"RTSEG_CONV_MFMA": "1", "RTSEG_CONV_WRES": "0"}):
        for k in ("RTSEG_CONV_MFMA", "RTSEG_CONV_HALO", "RTSEG_CONV_WRES", "RTSEG_DISABLE_HIP"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        calls.append(set())
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
    assert {"conv_wres", "conv_wres_dgrad"} <= calls[0], calls[0]
    assert not {"conv_wres", "conv_wres_dgrad"} & calls[1], calls[1]


# weight-gradient geometries (n, cin, h, w, cout) of 3x3 / stride-1 / pad-1 convs
WGRAD = [(2, 64, 17, 70, 64), (3, 128, 9, 40, 64), (1, 64, 6, 33, 192), (8, 64, 66, 256, 64), (2, 128, 16, 64, 128)]


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("geom", WGRAD)
@pytest.mark.parametrize("channels_last", [False, True])
def test_whalo_wgrad(geom, channels_last, variant):
    """Halo-tiled weight gradient (csrc/kernels/conv_whalo.hip) vs fp32 PyTorch on the same bf16
    operands: partial tiles, several channel pairs, split-K over many tiles (two-stage slab
    reduction), both parameter layouts; deterministic.  Variant 2: both output tiles per wave,
    the tile's K sub-steps split across the two wave halves and summed through LDS."""
    n, cin, h, w, cout = geom
    g = torch.Generator().manual_seed(4)
    cl = dict(memory_format=torch.channels_last)
    x = _t((n, cin, h, w), g).contiguous(**cl)
    dy = _t((n, cout, h, w), g).contiguous(**cl)
    dw = torch.ops.rtseg.conv_whalo_wgrad(x, dy, 3, 3, [1, 1], [1, 1], [1, 1], channels_last, variant)
    ref = torch.nn.grad.conv2d_weight(x.float(), (cout, cin, 3, 3), dy.float(), 1, 1, 1)
    assert dw.shape == ref.shape and dw.dtype == torch.float32
    assert dw.is_contiguous(memory_format=torch.channels_last) == channels_last or cin == 1
    f32_close(dw, ref)
    assert torch.equal(torch.ops.rtseg.conv_whalo_wgrad(x, dy, 3, 3, [1, 1], [1, 1], [1, 1], channels_last, variant), dw)


# register-weight halo conv (csrc/kernels/conv_hreg.hip): (n, cin, h, w, cout), Cin % 64, Cout % 128
HREG = [(2, 64, 9, 70, 128), (1, 128, 17, 130, 128), (3, 192, 6, 40, 256), (8, 128, 66, 256, 128)]


@pytest.mark.parametrize("rpw", [1, 2, 4, 5])
@pytest.mark.parametrize("geom", HREG)
def test_hreg_forward_and_stats(geom, rpw):
    n, cin, h, w, cout = geom
    g = torch.Generator().manual_seed(6)
    x = _t((n, cin, h, w), g).contiguous(memory_format=torch.channels_last)
    wt = _t((cout, cin, 3, 3), g, 1 / (3 * cin ** 0.5))
    wk = wt.permute(0, 2, 3, 1).contiguous()
    y, part = torch.ops.rtseg.conv_hreg(x, wk, [1, 1], [1, 1], [1, 1], True, rpw)
    ref = F.conv2d(x.float(), wt.float(), None, 1, 1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    bf16_close(y, ref)
    rf = ref.double()
    torch.testing.assert_close(part[:, :cout].double().sum(0), rf.sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[:, cout:].double().sum(0), rf.square().sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    y1, p1 = torch.ops.rtseg.conv_hreg(x, wk, [1, 1], [1, 1], [1, 1], True, rpw)
    assert torch.equal(y1, y) and torch.equal(p1, part)
    y2, _ = torch.ops.rtseg.conv_hreg(x, wk, [1, 1], [1, 1], [1, 1], False, rpw)
    assert torch.equal(y2, y)


@pytest.mark.parametrize("rpw", [1, 2, 4, 5])
@pytest.mark.parametrize("geom", HREG)
@pytest.mark.parametrize("with_addend", [False, True, "masked"])
def test_hreg_dgrad(geom, with_addend, rpw):
    """Data gradient of the forward conv (n, cout -> cin roles swapped: the dgrad reduces over the
    forward Cout and produces the forward Cin, so geometry (n, a, h, w, b) tests a conv b -> a)."""
    n, cout_fwd, h, w, cin_fwd = geom
    g = torch.Generator().manual_seed(8)
    cl = dict(memory_format=torch.channels_last)
    wt = _t((cout_fwd, cin_fwd, 3, 3), g, 1 / (3 * cout_fwd ** 0.5))
    dy = _t((n, cout_fwd, h, w), g).contiguous(**cl)
    add = _t((n, cin_fwd, h, w), g).contiguous(**cl)
    bits = _mask_bits(add.shape, 4)
    dx = torch.ops.rtseg.conv_hreg_dgrad(dy, wt.permute(1, 2, 3, 0).contiguous(), [n, cin_fwd, h, w], [1, 1], [1, 1],
                                         [1, 1], add if with_addend else None, rpw,
                                         bits if with_addend == "masked" else None)
    ref = torch.nn.grad.conv2d_input((n, cin_fwd, h, w), wt.float(), dy.float(), 1, 1, 1)
    bf16_close(dx, ref + _addend_ref(add, bits, with_addend))
