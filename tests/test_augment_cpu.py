"""GPU-augmentation host side on CPU (ops/augment.py): the parameter draw consumes the same
random stream as the CPU pipeline, the PyTorch formulation matches the numpy pipeline where
both resample identically, and a ``gpu_aug`` loader feeds the trainer's device path.
Reference: datasets/cityscapes.py:115-124 (albumentations training pipeline)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd.datasets import Cityscapes, get_loader
from realtime_semantic_segmentation_pytorch_amd.datasets import transforms as T
from realtime_semantic_segmentation_pytorch_amd.ops import augment as A

from test_user_surfaces_cpu import _aug_cfg, _fake_cityscapes


@pytest.fixture(autouse=True)
def _single_process(monkeypatch):
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)


def _pipeline(crop=32, randscale=(-0.5, 1.0), jitter=0.5, hue=0.2, flip=0.5, p=0.5):
    return T.Compose([T.Scale(1.0), T.RandomScale(list(randscale)), T.PadIfNeeded(crop, crop, 114, 0),
                      T.RandomCrop(crop, crop), T.ColorJitter(jitter, jitter, jitter, hue, p=p),
                      T.HorizontalFlip(flip), T.Normalize()])


@pytest.mark.parametrize("seed", range(6))
def test_draw_params_consumes_the_cpu_pipelines_stream(seed):
    tr = _pipeline()
    img = np.random.default_rng(seed).integers(0, 255, (40, 60, 3), dtype=np.uint8)
    msk = np.zeros((40, 60), np.uint8)
    r_cpu, r_gpu = np.random.default_rng(seed), np.random.default_rng(seed)
    out, _ = tr(img, msk, r_cpu)
    p, spec = A.draw_params(tr, 40, 60, r_gpu)
    assert r_cpu.random() == r_gpu.random()  # both consumed exactly the same draws
    assert (spec.crop_h, spec.crop_w) == (32, 32) and out.shape[:2] == (32, 32)
    assert p.shape == (A.NPARAMS,) and 0 <= p[A.NOPS] <= 4


def _cpu_pipeline_no_resize(img, msk, params, spec):
    """numpy CPU path with the drawn parameters applied by the transforms themselves."""
    tr = _pipeline()
    x, m = img, msk
    x, m = T.PadIfNeeded(spec.crop_h, spec.crop_w, 114, 0)(x, m, None)
    cy, cx = int(params[A.CY]), int(params[A.CX])
    x, m = x[cy:cy + spec.crop_h, cx:cx + spec.crop_w], m[cy:cy + spec.crop_h, cx:cx + spec.crop_w]
    if params[A.NOPS]:
        z = x.astype(np.float32) / 255.0
        seq = [(int(params[A.CODE]) >> (2 * k)) & 3 for k in range(int(params[A.NOPS]))]
        cm = 0.0
        for op in seq:
            if op == A.OP_BRIGHT:
                z = np.clip(z * params[A.BRIGHT], 0, 1)
            elif op == A.OP_CONTRAST:
                cm = (z @ np.float32([0.299, 0.587, 0.114])).mean()
                z = np.clip((z - cm) * params[A.CONTRAST] + cm, 0, 1)
            elif op == A.OP_SAT:
                g = (z @ np.float32([0.299, 0.587, 0.114]))[..., None]
                z = np.clip(g + (z - g) * params[A.SAT], 0, 1)
            else:
                h, s, v = T._rgb_to_hsv(z)
                z = T._hsv_to_rgb((h + params[A.HUE]) % 1.0, s, v).astype(np.float32)
        x = (z * 255.0 + 0.5).clip(0, 255).astype(np.uint8)
    if params[A.FLIP]:
        x, m = x[:, ::-1], m[:, ::-1]
    x, _ = tr.transforms[-1](x, None, None)
    return x, m


@pytest.mark.parametrize("seed", range(8))
def test_reference_matches_numpy_pipeline_without_resize(seed):
    rng = np.random.default_rng(100 + seed)
    h, w = (24, 40) if seed % 2 else (48, 50)  # smaller than the crop -> centred pad
    img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    msk = rng.integers(0, 34, (h, w), dtype=np.uint8)
    tr = _pipeline(randscale=(0.0, 0.0), p=1.0)
    params, spec = A.draw_params(tr, h, w, np.random.default_rng(seed))
    ref_img, ref_msk = _cpu_pipeline_no_resize(img, msk, params, spec)
    lut = torch.from_numpy(Cityscapes._lut.copy())
    out, mo = A.augment_reference(torch.from_numpy(img)[None], torch.from_numpy(msk)[None],
                                  torch.from_numpy(params)[None], lut, spec)
    got = out[0].permute(1, 2, 0).numpy()
    step = 1.0 / 255.0 / np.float32(T.IMAGENET_STD).min()
    diff = np.abs(got - ref_img)
    assert diff.max() <= step * 1.01, diff.max()  # at most one uint8 level (fp32 rounding ties)
    assert (diff > 1e-4).mean() < 0.01
    assert torch.equal(mo[0], torch.from_numpy(Cityscapes._lut[ref_msk]).to(torch.int64))


def test_reference_resize_is_bilinear_half_pixel_and_nearest_floor():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (30, 50, 3), dtype=np.uint8)
    msk = rng.integers(0, 19, (30, 50), dtype=np.uint8)
    p = np.zeros(A.NPARAMS, np.float32)
    p[A.NH], p[A.NW] = 45, 70
    p[A.BRIGHT] = p[A.CONTRAST] = p[A.SAT] = 1
    spec = A.AugmentSpec(45, 70, (0, 0, 0), (1, 1, 1))
    out, mo = A.augment_reference(torch.from_numpy(img)[None], torch.from_numpy(msk)[None], torch.from_numpy(p)[None],
                                  torch.arange(256, dtype=torch.uint8), spec)
    want = F.interpolate(torch.from_numpy(img).permute(2, 0, 1)[None].float(), size=(45, 70), mode="bilinear",
                         align_corners=False).round().clamp(0, 255) / 255.0
    assert torch.allclose(out, want, atol=1.01 / 255)
    ys = (torch.arange(45).float() * (30 / 45)).floor().long()
    xs = (torch.arange(70).float() * (50 / 70)).floor().long()
    assert torch.equal(mo[0], torch.from_numpy(msk).long()[ys][:, xs])


def test_pipeline_without_normalize_or_with_square_resize_is_rejected():
    with pytest.raises(ValueError):
        A.draw_params(T.Compose([T.RandomCrop(4, 4)]), 8, 8, np.random.default_rng(0))
    with pytest.raises(NotImplementedError):
        A.draw_params(T.Compose([T.ResizeToSquare(8), T.Normalize()]), 8, 8, np.random.default_rng(0))


def test_gpu_aug_loader_feeds_trainer_device_path(tmp_path):
    _fake_cityscapes(tmp_path, n=4)
    cfg = _aug_cfg(tmp_path, gpu_aug=True)
    ds = Cityscapes(cfg, "train")
    img, msk, prm = ds[(1, 3)]
    assert img.dtype == torch.uint8 and img.shape == (48, 96, 3) and msk.shape == (48, 96)
    assert prm.shape == (A.NPARAMS,) and (ds.aug_spec.crop_h, ds.aug_spec.crop_w) == (32, 32)
    # the same (seed, epoch, index) draws the same parameters as the CPU path's stream
    p2, _ = A.draw_params(ds.transform, 48, 96, np.random.default_rng([cfg.random_seed, 3, 1]))
    assert np.array_equal(prm.numpy(), p2)
    train_loader, _ = get_loader(cfg)
    batch = next(iter(train_loader))
    assert len(batch) == 3
    x, y = A.augment_batch(*batch, ds.aug_lut, ds.aug_spec)
    assert x.shape == (2, 3, 32, 32) and y.shape == (2, 32, 32) and y.dtype == torch.int64
    assert torch.isfinite(x).all() and ((y < 19) | (y == 255)).all()
