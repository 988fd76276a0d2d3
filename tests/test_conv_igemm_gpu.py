"""32x32x16-MFMA implicit-GEMM conv family (csrc/kernels/conv_igemm.hip) vs fp32 PyTorch:
forward (+ BN-statistics slab, + inference BN/residual/act epilogue), data gradient (tap-table /
sub-pixel phases for strided convs) and weight gradient (split-K over pixels)."""
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

# (n, cin, h, w, cout, k, stride, dilation) -- odd sizes, partial tiles, strides, dilation
GEOMS = [
    (2, 64, 17, 23, 64, 3, 1, 1),
    (2, 64, 32, 40, 128, 3, 2, 1),
    (1, 128, 9, 14, 200, 3, 1, 2),
    (3, 128, 16, 16, 64, 1, 1, 1),
    (1, 64, 7, 5, 24, 5, 1, 1),
    (2, 256, 12, 20, 256, 3, 1, 1),
    (2, 128, 15, 21, 128, 1, 2, 1),
    (1, 192, 11, 13, 320, 3, 2, 1),
]
# big enough that the persistent grid walks several M tiles per block (the BN statistics are
# summed over a block's tiles before the one slab row per block is written), per tile config
BIG_GEOMS = [
    (8, 64, 128, 256, 64, 3, 1, 1),    # 512 x 64 tiles
    (16, 128, 128, 128, 128, 3, 1, 1),  # 512 x 128
    (16, 256, 64, 128, 256, 3, 1, 1),   # 256 x 256
    (8, 64, 96, 128, 200, 3, 1, 1),     # 256 x 256, partial channel tile
]


@pytest.fixture(autouse=True)
def _lib():
    assert ops.load(), "HIP extension must load on the GPU box"


def _case(n, cin, h, w, cout, k, s, d, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(n, cin, h, w, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5).to(DEV, torch.bfloat16)
    return x, wt


def _close(got, ref, tol):
    torch.testing.assert_close(got.float(), ref, atol=tol * ref.abs().max().item() + 1e-6, rtol=tol)


@pytest.mark.parametrize("geom", GEOMS + BIG_GEOMS)
def test_igemm_forward_and_stats(geom):
    n, cin, h, w, cout, k, s, d = geom
    x, wt = _case(*geom)
    p = (k - 1) // 2 * d
    y, part = torch.ops.rtseg.conv_igemm(x, wt.permute(0, 2, 3, 1).contiguous(), [s, s], [p, p], [d, d], True,
                                         None, None, 0)
    ref = F.conv2d(x.float(), wt.float(), None, s, p, d)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    bf16_close(y, ref)
    # the slab holds the statistics of the fp32 conv outputs (the kernel's accumulators)
    rf = ref.double()
    assert part.shape[0] <= 256 and part.shape[1] == 2 * cout
    torch.testing.assert_close(part[:, :cout].double().sum(0), rf.sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[:, cout:].double().sum(0), rf.square().sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    # deterministic: a second launch gives the same bits
    _, part2 = torch.ops.rtseg.conv_igemm(x, wt.permute(0, 2, 3, 1).contiguous(), [s, s], [p, p], [d, d], True,
                                          None, None, 0)
    assert torch.equal(part, part2)


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("with_res", [False, True])
def test_igemm_bn_epilogue(act, with_res):
    n, cin, h, w, cout, k = 2, 64, 20, 24, 128, 3
    x, wt = _case(n, cin, h, w, cout, k, 1, 1, seed=3)
    ss = torch.cat([torch.rand(cout, device=DEV) + 0.5, torch.randn(cout, device=DEV)]).contiguous()
    res = None
    if with_res:
        res = torch.randn(n, cout, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y, _ = torch.ops.rtseg.conv_igemm(x, wt.permute(0, 2, 3, 1).contiguous(), [1, 1], [1, 1], [1, 1], False,
                                      ss, res, act)
    ref = F.conv2d(x.float(), wt.float(), None, 1, 1) * ss[:cout].view(1, -1, 1, 1) + ss[cout:].view(1, -1, 1, 1)
    if with_res:
        ref = ref + res.float()
    if act == 1:
        ref = ref.relu()
    elif act == 2:
        ref = ref.clamp(0, 6)
    bf16_close(y, ref)


@pytest.mark.parametrize("geom", [(1, 256, 16, 32, 256, 3, 1, 1), (1, 512, 8, 16, 512, 3, 1, 1),
                                  (1, 128, 33, 20, 256, 3, 2, 1), (2, 64, 9, 13, 72, 1, 1, 1)])
@pytest.mark.parametrize("with_res", [False, True])
@pytest.mark.parametrize("split_k", [False, True])
def test_igemm_small_tiles_inference(geom, with_res, split_k):
    """The 128 x 64-tile, 2-blocks-per-CU configuration (conv_igemm_small: batch-1 inference)
    against fp32, and bitwise against the shape-picked tiles (same K order per output); with
    split_k the layers with < 256 tiles sum K parts in fp32 and apply the BN epilogue after
    (every geometry here but the last splits)."""
    n, cin, h, w, cout, k, s, d = geom
    x, wt = _case(*geom, seed=13)
    p = (k - 1) // 2 * d
    g = torch.Generator().manual_seed(14)
    ss = torch.cat([torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g)]).to(DEV).contiguous()
    ho, wo = (h + 2 * p - d * (k - 1) - 1) // s + 1, (w + 2 * p - d * (k - 1) - 1) // s + 1
    res = None
    if with_res:
        res = torch.randn(n, cout, ho, wo, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wk = wt.permute(0, 2, 3, 1).contiguous()
    y = torch.ops.rtseg.conv_igemm_small(x, wk, [s, s], [p, p], [d, d], ss, res, 1, split_k)
    ref = F.conv2d(x.float(), wt.float(), None, s, p, d) * ss[:cout].view(1, -1, 1, 1) + ss[cout:].view(1, -1, 1, 1)
    if with_res:
        ref = ref + res.float()
    bf16_close(y, ref.relu())
    assert torch.equal(y, torch.ops.rtseg.conv_igemm_small(x, wk, [s, s], [p, p], [d, d], ss, res, 1, split_k))
    if not split_k:
        y0, _ = torch.ops.rtseg.conv_igemm(x, wk, [s, s], [p, p], [d, d], False, ss, res, 1)
        assert torch.equal(y, y0)


DGRAD = [
    (2, 64, 17, 23, 64, 3, 1, 1),
    (2, 64, 32, 40, 128, 3, 2, 1),
    (2, 48, 33, 41, 128, 3, 2, 1),   # odd input: the last phase rows are partial
    (1, 128, 9, 14, 192, 3, 1, 2),
    (3, 128, 16, 16, 64, 1, 1, 1),
    (2, 64, 15, 21, 128, 1, 2, 1),   # 1x1 stride 2: three of four phases have no tap (zeros)
    (1, 24, 7, 9, 64, 5, 1, 1),
]


@pytest.mark.parametrize("geom", DGRAD)
def test_igemm_dgrad(geom):
    n, cin, h, w, cout, k, s, d = geom
    x, wt = _case(*geom, seed=7)
    p = (k - 1) // 2 * d
    ho = (h + 2 * p - d * (k - 1) - 1) // s + 1
    wo = (w + 2 * p - d * (k - 1) - 1) // s + 1
    dy = torch.randn(n, cout, ho, wo, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dx = torch.ops.rtseg.conv_igemm_dgrad(dy, wt.permute(1, 2, 3, 0).contiguous(), list(x.shape), [s, s], [p, p],
                                          [d, d])
    ref = torch.nn.grad.conv2d_input(x.shape, wt.float(), dy.float(), s, p, d)
    assert dx.shape == x.shape and dx.is_contiguous(memory_format=torch.channels_last)
    bf16_close(dx, ref)


WGRAD = [
    (2, 64, 17, 23, 64, 3, 1, 1),
    (2, 64, 32, 40, 128, 3, 2, 1),
    (1, 128, 9, 14, 192, 3, 1, 2),
    (3, 128, 16, 16, 64, 1, 1, 1),
    (2, 128, 15, 21, 256, 1, 2, 1),
    (1, 64, 7, 9, 128, 5, 1, 1),
    (4, 256, 32, 48, 256, 3, 1, 1),
]


@pytest.mark.parametrize("geom", WGRAD)
def test_igemm_wgrad(geom):
    n, cin, h, w, cout, k, s, d = geom
    x, wt = _case(*geom, seed=11)
    p = (k - 1) // 2 * d
    ho = (h + 2 * p - d * (k - 1) - 1) // s + 1
    wo = (w + 2 * p - d * (k - 1) - 1) // s + 1
    dy = torch.randn(n, cout, ho, wo, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dw = torch.ops.rtseg.conv_igemm_wgrad(x, dy, k, k, [s, s], [p, p], [d, d])
    ref = torch.nn.grad.conv2d_weight(x.float(), wt.shape, dy.float(), s, p, d)
    assert dw.shape == wt.shape and dw.dtype == torch.float32 and dw.is_contiguous()
    f32_close(dw, ref)


def _handoff_nodes(out):
    seen, stack, hit = set(), [out.grad_fn], 0
    while stack:
        fn = stack.pop()
        if fn is None or id(fn) in seen:
            continue
        seen.add(id(fn))
        hit += isinstance(getattr(fn, "addend_slot", None), list)
        stack.extend(f for f, _ in fn.next_functions)
    return hit


@pytest.mark.parametrize("with_addend", [False, True, "masked"])
def test_igemm_dgrad_addend(with_addend):
    x, wt = _case(2, 64, 17, 23, 64, 3, 2, 1, seed=5)
    dy = torch.randn(2, 64, 9, 12, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    add = torch.randn(x.shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    bits = _mask_bits(x.shape, 6)
    dx = torch.ops.rtseg.conv_igemm_dgrad(dy, wt.permute(1, 2, 3, 0).contiguous(), list(x.shape), [2, 2], [1, 1],
                                          [1, 1], None, add if with_addend else None,
                                          bits if with_addend == "masked" else None)
    ref = torch.nn.grad.conv2d_input(x.shape, wt.float(), dy.float(), 2, 1, 1)
    bf16_close(dx, ref + _addend_ref(add, bits, with_addend))


def test_residual_grad_handoff_matches_plain_add(monkeypatch):
    """A chain of DDRNet RBs: each RB tail hands its residual gradient to the next-upstream conv's
    dgrad epilogue (ops/bn.py); the gradients must match the autograd accumulation."""
    from realtime_semantic_segmentation_pytorch_amd.models.ddrnet import RB
    from realtime_semantic_segmentation_pytorch_amd.ops import bn as bn_mod

    monkeypatch.setenv("RTSEG_CONV_MFMA", "1")
    torch.manual_seed(0)
    net = ops.convert_batchnorm(torch.nn.Sequential(RB(64, 64), RB(64, 64), RB(64, 64))).to(DEV)
    net = net.to(memory_format=torch.channels_last).train()
    x0 = torch.randn(2, 64, 24, 40, device=DEV).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(2, 64, 24, 40, device=DEV)
    res = {}
    for on in ("masked", True, False):
        monkeypatch.setattr(bn_mod, "_HANDOFF", bool(on))
        monkeypatch.setattr(bn_mod, "_MASKED_HANDOFF", on == "masked")
        before = bn_mod.MASKED_HANDOFFS[0]
        net.zero_grad(set_to_none=True)
        x = x0.to(torch.bfloat16).requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = net(x)
        nodes = _handoff_nodes(y)
        (y.float() * gy).sum().backward()
        res[on] = (nodes, x.grad.float().clone(),
                   {n: p.grad.float().clone() for n, p in net.named_parameters() if p.grad is not None})
        assert (bn_mod.MASKED_HANDOFFS[0] > before) == (on == "masked")
    assert res[True][0] >= 2 and res[False][0] == 0
    # the masked hand-off adds exactly the values the written-out residual gradient held (g or 0)
    assert torch.equal(res["masked"][1], res[True][1])
    for n, g in res[True][2].items():
        assert torch.equal(res["masked"][2][n], g), n
    _close(res[True][1], res[False][1], 2e-2)
    for n, g in res[False][2].items():
        _close(res[True][2][n], g, 2e-2)


@pytest.mark.parametrize("shape", [(2, 64, 17, 23, 128), (1, 128, 16, 32, 64)])
@pytest.mark.parametrize("with_addend", [False, True])
def test_igemm_dgrad_phase_addend(shape, with_addend):
    """Stride-2 3 x 3 dgrad with a phase-(0, 0) addend: added to exactly the even rows / columns
    of dx (odd sizes: the last phase-(0, 0) row / column included), on top of a full addend."""
    n, cin, h, w, cout = shape
    x, wt = _case(n, cin, h, w, cout, 3, 2, 1, seed=9)
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    cl = dict(memory_format=torch.channels_last)
    dy = torch.randn(n, cout, ho, wo, device=DEV).to(torch.bfloat16).contiguous(**cl)
    add = torch.randn(x.shape, device=DEV).to(torch.bfloat16).contiguous(**cl)
    ph = torch.randn(n, cin, (h + 1) // 2, (w + 1) // 2, device=DEV).to(torch.bfloat16).contiguous(**cl)
    dx = torch.ops.rtseg.conv_igemm_dgrad(dy, wt.permute(1, 2, 3, 0).contiguous(), list(x.shape), [2, 2], [1, 1],
                                          [1, 1], None, add if with_addend else None, None, ph)
    ref = torch.nn.grad.conv2d_input(x.shape, wt.float(), dy.float(), 2, 1, 1)
    if with_addend:
        ref = ref + add.float()
    ref[:, :, ::2, ::2] += ph.float()
    bf16_close(dx, ref)
    with pytest.raises(RuntimeError, match="phase_addend"):
        torch.ops.rtseg.conv_igemm_dgrad(dy, wt.permute(1, 2, 3, 0).contiguous(), list(x.shape), [2, 2], [1, 1],
                                         [1, 1], None, None, None, ph[:, :, 1:])


def test_skip_grad_handoff_bilateral_fusion(monkeypatch):
    """DDRNet's bilateral fusion: x_high feeds both the fusion's 3 x 3 conv and the skip of the
    upsample-add.  The upsample node hands the skip gradient to the conv's dgrad epilogue
    (ops/interp.py, ops/conv.py consumer_for) when the conv has not run yet; gradients match the
    autograd accumulation, and the hand-off really happened."""
    from realtime_semantic_segmentation_pytorch_amd.models.ddrnet import BilateralFusion
    from realtime_semantic_segmentation_pytorch_amd.ops import interp as interp_mod

    torch.manual_seed(0)
    net = ops.convert_batchnorm(BilateralFusion(256, 128, 2)).to(DEV).to(memory_format=torch.channels_last).train()
    lo0 = torch.randn(2, 256, 12, 20, device=DEV).contiguous(memory_format=torch.channels_last)
    hi0 = torch.randn(2, 128, 24, 40, device=DEV).contiguous(memory_format=torch.channels_last)
    g_lo = torch.randn(2, 256, 12, 20, device=DEV)
    g_hi = torch.randn(2, 128, 24, 40, device=DEV)
    res = {}
    for on in (True, False):
        monkeypatch.setattr(interp_mod, "_SKIP_HANDOFF", on)
        before = interp_mod.SKIP_HANDOFFS[0]
        net.zero_grad(set_to_none=True)
        lo = lo0.to(torch.bfloat16).requires_grad_(True)
        hi = hi0.to(torch.bfloat16).requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            a, b = net(lo, hi)
        ((a.float() * g_lo).sum() + (b.float() * g_hi).sum()).backward()
        res[on] = (interp_mod.SKIP_HANDOFFS[0] - before, lo.grad.float().clone(), hi.grad.float().clone(),
                   {n: p.grad.float().clone() for n, p in net.named_parameters()})
    assert res[True][0] == 1 and res[False][0] == 0
    for k in (1, 2):
        _close(res[True][k], res[False][k], 1e-2)
    for n, g in res[False][3].items():
        _close(res[True][3][n], g, 1e-2)


@pytest.mark.parametrize("case", [
    (2, 64, 16, 24, 64, 3, 2, 1),     # 3 x 3 / 2: phases of 1, 2, 2, 4 taps (null-tap padding)
    (2, 128, 32, 16, 128, 3, 2, 1),
    (2, 64, 24, 32, 128, 3, 4, 1),    # 3 x 3 / 4 (DDRNet's x4 fusion): 16 phases, 7 of them empty
    (2, 64, 16, 16, 128, 1, 2, 0),    # 1 x 1 / 2 shortcut: 1 phase with a tap, 3 all-null
    (3, 32, 40, 48, 64, 3, 2, 1),     # Cin 32 (16-byte rows), tiles past M
])
@pytest.mark.parametrize("extras", ["none", "addend", "phase_addend"])
def test_igemm_dgrad_fused_phases(case, extras):
    """Data gradient of a strided conv with every output phase in one launch (fused_phases=True)
    against the fp32 reference and against the per-phase launches (same accumulation order per
    output pixel: bitwise equal)."""
    n, cin, h, w, cout, k, s, p = case
    x, wt = _case(n, cin, h, w, cout, k, s, 1, seed=21)
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    cl = dict(memory_format=torch.channels_last)
    g = torch.Generator(device="cpu").manual_seed(22)
    dy = torch.randn(n, cout, ho, wo, generator=g).to(DEV, torch.bfloat16).contiguous(**cl)
    add = torch.randn(x.shape, generator=g).to(DEV, torch.bfloat16).contiguous(**cl) if extras == "addend" else None
    ph = (torch.randn(n, cin, h // s, w // s, generator=g).to(DEV, torch.bfloat16).contiguous(**cl)
          if extras == "phase_addend" else None)
    wtr = wt.permute(1, 2, 3, 0).contiguous()
    args = (dy, wtr, list(x.shape), [s, s], [p, p], [1, 1], None, add, None, ph)
    fused = torch.ops.rtseg.conv_igemm_dgrad(*args, True)
    split = torch.ops.rtseg.conv_igemm_dgrad(*args, False)
    ref = torch.nn.grad.conv2d_input(x.shape, wt.float(), dy.float(), s, p, 1)
    if add is not None:
        ref = ref + add.float()
    if ph is not None:
        ref[:, :, ::s, ::s] += ph.float()
    bf16_close(fused, ref)
    assert torch.equal(fused, split)


def test_igemm_dgrad_fused_phases_rejects():
    x, wt = _case(1, 64, 15, 16, 64, 3, 2, 1)  # H % 2 != 0
    dy = torch.randn(1, 64, 8, 8, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with pytest.raises(RuntimeError, match="fused phases"):
        torch.ops.rtseg.conv_igemm_dgrad(dy, wt.permute(1, 2, 3, 0).contiguous(), list(x.shape), [2, 2], [1, 1],
                                         [1, 1], None, None, None, None, True)
