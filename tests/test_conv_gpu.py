"""MFMA implicit-GEMM conv (csrc/kernels/conv_mfma.hip) vs F.conv2d in fp32."""
import pytest
import torch
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (n, cin, h, w, cout, k, stride, dilation)
GEOMS = [
    (2, 32, 17, 23, 16, 3, 1, 1),
    (2, 64, 32, 40, 128, 3, 2, 1),
    (1, 96, 9, 14, 200, 3, 1, 2),
    (3, 128, 16, 16, 64, 1, 1, 1),
    (1, 64, 7, 5, 24, 5, 1, 1),
    (2, 256, 12, 20, 256, 3, 1, 1),
]


@pytest.fixture(autouse=True)
def _lib():
    assert ops.load(), "HIP extension must load on the GPU box"


def _case(n, cin, h, w, cout, k, s, d, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(n, cin, h, w, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5).to(DEV, torch.bfloat16)
    return x, wt


@pytest.mark.parametrize("geom", GEOMS)
def test_conv_mfma_matches_conv2d(geom):
    n, cin, h, w, cout, k, s, d = geom
    x, wt = _case(*geom)
    p = (k - 1) // 2 * d
    y, part = torch.ops.rtseg.conv_mfma(x, wt.permute(0, 2, 3, 1).contiguous(), [s, s], [p, p], [d, d], True,
                                        None, None, 0)
    ref = F.conv2d(x.float(), wt.float(), None, s, p, d)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, atol=2e-2 * ref.abs().max().item(), rtol=2e-2)
    # BN statistics epilogue: per-channel sum / sum of squares of the bf16 outputs
    yf = y.float()
    s1 = part[:, :cout].double().sum(0)
    s2 = part[:, cout:].double().sum(0)
    torch.testing.assert_close(s1, yf.double().sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s2, yf.double().square().sum((0, 2, 3)), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("with_res", [False, True])
def test_conv_mfma_bn_epilogue(act, with_res):
    n, cin, h, w, cout, k = 2, 64, 20, 24, 64, 3
    x, wt = _case(n, cin, h, w, cout, k, 1, 1, seed=3)
    ss = torch.cat([torch.rand(cout, device=DEV) + 0.5, torch.randn(cout, device=DEV)]).contiguous()
    res = None
    if with_res:
        res = torch.randn(n, cout, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y, _ = torch.ops.rtseg.conv_mfma(x, wt.permute(0, 2, 3, 1).contiguous(), [1, 1], [1, 1], [1, 1], False,
                                     ss, res, act)
    ref = F.conv2d(x.float(), wt.float(), None, 1, 1) * ss[:cout].view(1, -1, 1, 1) + ss[cout:].view(1, -1, 1, 1)
    if with_res:
        ref = ref + res.float()
    if act == 1:
        ref = ref.relu()
    torch.testing.assert_close(y.float(), ref, atol=3e-2 * ref.abs().max().item(), rtol=3e-2)
