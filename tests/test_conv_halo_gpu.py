"""Halo-tiled stride-1 conv (csrc/kernels/conv_halo.hip) vs fp32 PyTorch: forward (+ BN-statistics
slab, + inference BN / residual / act epilogue) and data gradient (+ residual-gradient addend),
on partial tiles (H % 4, W % 64), several 64-channel chunks, partial 128-channel output tiles,
and a valid (unpadded) 3x3; 3-tap convs are rejected (their halo cannot ride on the taps)."""
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

# (n, cin, h, w, cout, kh, kw, ph, pw)
GEOMS = [
    (2, 64, 17, 70, 64, 3, 3, 1, 1),
    (2, 128, 9, 130, 128, 3, 3, 1, 1),
    (1, 256, 6, 40, 192, 3, 3, 1, 1),
    (3, 64, 8, 64, 320, 3, 3, 1, 1),
    (1, 64, 10, 69, 128, 3, 3, 0, 0),
]
# several tiles per block of the persistent grid (BN statistics summed per block before its one
# slab row is written): 64- and 128-channel configs, a partial last tile row
BIG_GEOMS = [
    (8, 64, 130, 256, 64, 3, 3, 1, 1),
    (8, 128, 66, 256, 128, 3, 3, 1, 1),
]


@pytest.fixture(autouse=True)
def _lib():
    assert ops.load(), "HIP extension must load on the GPU box"


def _case(n, cin, h, w, cout, kh, kw, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(n, cin, h, w, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cout, cin, kh, kw, generator=g) / (cin * kh * kw) ** 0.5).to(DEV, torch.bfloat16)
    return x, wt


def _close(got, ref, tol):
    torch.testing.assert_close(got.float(), ref, atol=tol * ref.abs().max().item() + 1e-6, rtol=tol)


@pytest.mark.parametrize("geom", GEOMS + BIG_GEOMS)
def test_halo_forward_and_stats(geom):
    n, cin, h, w, cout, kh, kw, ph, pw = geom
    x, wt = _case(n, cin, h, w, cout, kh, kw)
    wk = wt.permute(0, 2, 3, 1).contiguous()
    y, part = torch.ops.rtseg.conv_halo(x, wk, [1, 1], [ph, pw], [1, 1], True, None, None, 0)
    ref = F.conv2d(x.float(), wt.float(), None, 1, (ph, pw))
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    bf16_close(y, ref)
    rf = ref.double()  # the slab holds the statistics of the fp32 outputs (the accumulators)
    torch.testing.assert_close(part[:, :cout].double().sum(0), rf.sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[:, cout:].double().sum(0), rf.square().sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    assert part.shape[0] <= 256
    _, p1 = torch.ops.rtseg.conv_halo(x, wk, [1, 1], [ph, pw], [1, 1], True, None, None, 0)
    assert torch.equal(p1, part)  # deterministic
    y2, p2 = torch.ops.rtseg.conv_halo(x, wk, [1, 1], [ph, pw], [1, 1], False, None, None, 0)
    assert p2 is None or p2.numel() == 0
    torch.testing.assert_close(y2, y, rtol=0, atol=0)


def test_halo_rejects_three_tap_convs():
    x, wt = _case(1, 64, 8, 64, 64, 3, 1)
    with pytest.raises(RuntimeError, match="conv_halo"):
        torch.ops.rtseg.conv_halo(x, wt.permute(0, 2, 3, 1).contiguous(), [1, 1], [1, 0], [1, 1], False, None,
                                  None, 0)


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("with_res", [False, True])
def test_halo_bn_epilogue(act, with_res):
    n, cin, h, w, cout = 2, 128, 10, 72, 128
    x, wt = _case(n, cin, h, w, cout, 3, 3, seed=4)
    g = torch.Generator(device="cpu").manual_seed(9)
    scale, shift = torch.randn(cout, generator=g).to(DEV), torch.randn(cout, generator=g).to(DEV)
    res = torch.randn(n, cout, h, w, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y, _ = torch.ops.rtseg.conv_halo(x, wt.permute(0, 2, 3, 1).contiguous(), [1, 1], [1, 1], [1, 1], False,
                                     torch.cat([scale, shift]), res if with_res else None, act)
    ref = F.conv2d(x.float(), wt.float(), None, 1, 1) * scale.view(1, -1, 1, 1) + shift.view(1, -1, 1, 1)
    if with_res:
        ref = ref + res.float()
    ref = ref.relu() if act == 1 else ref.clamp(0, 6) if act == 2 else ref
    bf16_close(y, ref)


@pytest.mark.parametrize("geom", GEOMS)
@pytest.mark.parametrize("with_addend", [False, True, "masked"])
def test_halo_dgrad(geom, with_addend):
    n, cin, h, w, cout, kh, kw, ph, pw = geom
    x, wt = _case(n, cin, h, w, cout, kh, kw, seed=2)
    ho, wo = h + 2 * ph - kh + 1, w + 2 * pw - kw + 1
    g = torch.Generator(device="cpu").manual_seed(5)
    cl = dict(memory_format=torch.channels_last)
    dy = torch.randn(n, cout, ho, wo, generator=g).to(DEV, torch.bfloat16).contiguous(**cl)
    add = torch.randn(x.shape, generator=g).to(DEV, torch.bfloat16).contiguous(**cl)
    if cout % 64 or cin % 64:
        pytest.skip("dgrad reduces over Cout and produces Cin: both must be 64-channel multiples")
    bits = _mask_bits(add.shape, 7)
    dx = torch.ops.rtseg.conv_halo_dgrad(dy, wt.permute(1, 2, 3, 0).contiguous(), list(x.shape), [1, 1], [ph, pw],
                                         [1, 1], add if with_addend else None, bits if with_addend == "masked" else None)
    ref = torch.nn.grad.conv2d_input(x.shape, wt.float(), dy.float(), 1, (ph, pw), 1)
    bf16_close(dx, ref + _addend_ref(add, bits, with_addend))


def test_halo_routed_training_step(monkeypatch):
    """DDRNet RB chain with the halo kernel forced first vs the gather kernel (both bf16 HIP
    paths): outputs and gradients agree up to bf16 rounding (relative Frobenius error -- a ReLU
    mask bit that flips on a 1-ulp difference moves single gradient elements by a whole dy)."""
    from realtime_semantic_segmentation_pytorch_amd.models.ddrnet import RB

    torch.manual_seed(0)
    net = ops.convert_batchnorm(torch.nn.Sequential(RB(64, 64), RB(64, 64))).to(DEV)
    net = net.to(memory_format=torch.channels_last).train()
    x0 = torch.randn(2, 64, 24, 72, device=DEV).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(2, 64, 24, 72, device=DEV)
    from realtime_semantic_segmentation_pytorch_amd.ops import conv as conv_mod

    calls = []

    class _Spy:  # records which rtseg ops the conv routing calls
        def __getattr__(self, name):
            calls[-1].add(name)
            return getattr(torch.ops.rtseg, name)

    spy = _Spy()
    monkeypatch.setattr(conv_mod, "ops", lambda: spy)
    grads = {}
    for env in ({"RTSEG_CONV_MFMA": "1", "RTSEG_CONV_HALO": "1"}, {"RTSEG_CONV_MFMA": "1", "RTSEG_CONV_HALO": "0"}):
        for k in ("RTSEG_CONV_MFMA", "RTSEG_CONV_HALO", "RTSEG_DISABLE_HIP"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        calls.append(set())
        net.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = net(x)
        (y.float() * gy).sum().backward()
        grads[len(grads)] = (y.float().detach(), x.grad.float().clone(),
                             {n: p.grad.float().clone() for n, p in net.named_parameters()})
    (y0, gx0, gp0), (y1, gx1, gp1) = grads[0], grads[1]

    def rel(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()

    assert rel(y0, y1) < 1e-2
    assert rel(gx0, gx1) < 2e-2
    for n, g in gp1.items():
        assert rel(gp0[n], g) < 3e-2, n
    assert {"conv_halo", "conv_halo_dgrad"} <= calls[0], calls[0]
    assert not {"conv_halo", "conv_halo_dgrad"} & calls[1], calls[1]
