"""GPU augmentation kernel (augment.hip) against its PyTorch formulation (ops/augment.py), which
the CPU tests pin to the numpy pipeline.  Reference: datasets/cityscapes.py:115-124."""
import numpy as np
import pytest
import torch

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.datasets import Cityscapes
from realtime_semantic_segmentation_pytorch_amd.datasets import transforms as T
from realtime_semantic_segmentation_pytorch_amd.ops import augment as A

pytestmark = pytest.mark.gpu


def _batch(n, h, w, crop, seed, randscale=(-0.5, 1.0), p=1.0):
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (n, h, w, 3), dtype=np.uint8)
    # smooth-ish images so bilinear rounding ties are rare but present
    msk = rng.integers(0, 34, (n, h, w), dtype=np.uint8)
    tr = T.Compose([T.Scale(1.0), T.RandomScale(list(randscale)), T.PadIfNeeded(crop[0], crop[1], 114, 0),
                    T.RandomCrop(*crop), T.ColorJitter(0.5, 0.5, 0.5, 0.2, p=p), T.HorizontalFlip(0.5),
                    T.Normalize()])
    rows, spec = [], None
    for i in range(n):
        prm, spec = A.draw_params(tr, h, w, np.random.default_rng([seed, 0, i]))
        rows.append(prm)
    return torch.from_numpy(img), torch.from_numpy(msk), torch.from_numpy(np.stack(rows)), spec


@pytest.mark.parametrize("seed,h,w,crop", [(0, 64, 128, (48, 96)), (1, 40, 60, (64, 64)), (2, 97, 131, (50, 70)),
                                           (3, 128, 256, (128, 128))])
def test_augment_kernel_matches_reference(seed, h, w, crop):
    assert ops.load()
    img, msk, prm, spec = _batch(4, h, w, crop, seed)
    assert A.has_contrast(prm) or seed > 0
    lut = torch.from_numpy(Cityscapes._lut.copy())
    ref_x, ref_y = A.augment_reference(img, msk, prm, lut, spec)
    x, y = A.augment_batch(img.cuda(), msk.cuda(), prm, lut, spec)
    torch.cuda.synchronize()
    step = 1.0 / 255.0 / min(spec.std)
    d = (x.cpu() - ref_x).abs()
    assert d.max() <= 2.01 * step, float(d.max())  # fp32 contraction may move a tie by one level
    assert (d > 1e-4).float().mean() < 0.005
    assert (y.cpu() != ref_y).float().mean() < 1e-3


def test_augment_kernel_bf16_channels_last_and_uint8_masks():
    img, msk, prm, spec = _batch(3, 80, 120, (64, 96), 7)
    lut = torch.from_numpy(Cityscapes._lut.copy())
    x32, y64 = A.augment_batch(img.cuda(), msk.cuda(), prm, lut, spec)
    xb, y8 = A.augment_batch(img.cuda(), msk.cuda(), prm, lut, spec, out_dtype=torch.bfloat16, channels_last=True,
                             mask_dtype=torch.uint8)
    assert xb.is_contiguous(memory_format=torch.channels_last) and xb.dtype == torch.bfloat16
    assert torch.allclose(xb.float(), x32, atol=0.02, rtol=0.01)
    assert torch.equal(y8.long(), y64)


def test_augment_kernel_without_jitter_is_exact():
    img, msk, prm, spec = _batch(2, 64, 64, (64, 64), 11, randscale=(0.0, 0.0), p=0.0)
    lut = torch.arange(256, dtype=torch.uint8)
    ref_x, ref_y = A.augment_reference(img, msk, prm, lut, spec)
    x, y = A.augment_batch(img.cuda(), msk.cuda(), prm, lut, spec)
    assert torch.allclose(x.cpu(), ref_x, atol=1e-5) and torch.equal(y.cpu(), ref_y)
