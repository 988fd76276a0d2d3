"""HIP PixelShuffle / PixelUnshuffle / channel shuffle (shuffle.hip) against PyTorch, forward and
backward, contiguous and channels-last.  Reference: models/farseenet.py:59,82,
models/modules.py:18-32."""
import pytest
import torch
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd import ops

pytestmark = pytest.mark.gpu


def _torch_cs(x, g):
    n, c, h, w = x.shape
    return x.reshape(n, g, c // g, h, w).transpose(1, 2).reshape(n, c, h, w)


CASES = [("ps", 2, (2, 32, 9, 13)), ("ps", 4, (1, 48, 5, 7)), ("pu", 2, (2, 6, 10, 14)), ("pu", 3, (1, 5, 9, 12)),
         ("cs", 2, (2, 64, 11, 17)), ("cs", 4, (3, 24, 8, 8)), ("cs", 3, (2, 48, 7, 5))]


@pytest.mark.parametrize("op,r,shape", CASES)
@pytest.mark.parametrize("cl", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_shuffle_matches_torch(op, r, shape, cl, dtype):
    assert ops.load()
    x = torch.randn(shape, device="cuda").to(dtype)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    hip = {"ps": ops.pixel_shuffle, "pu": ops.pixel_unshuffle, "cs": ops.channel_shuffle}[op]
    ref = {"ps": F.pixel_shuffle, "pu": F.pixel_unshuffle, "cs": _torch_cs}[op]
    xh, xr = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    yh, yr = hip(xh, r), ref(xr, r)
    assert torch.equal(yh, yr)
    assert yh.is_contiguous(memory_format=torch.channels_last) == cl or not cl
    g = torch.randn_like(yr)
    yh.backward(g)
    yr.backward(g)
    assert torch.equal(xh.grad, xr.grad)


def test_farseenet_pixel_shuffle_modules_are_converted():
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.models import get_model

    cfg = BaseConfig()
    cfg.model, cfg.num_class = "farseenet", 19
    m = get_model(cfg).cuda().to(memory_format=torch.channels_last)
    assert any(isinstance(mm, ops.shuffle.PixelShuffle) for mm in m.modules())
    x = torch.randn(2, 3, 128, 256, device="cuda").contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    y.float().mean().backward()
    assert y.shape[-2:] == (128, 256)
