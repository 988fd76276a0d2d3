"""GPU-side training augmentation (kernel: ``csrc/kernels/augment.hip``).

Reference: the albumentations training pipeline of datasets/cityscapes.py:115-124
(Scale, RandomScale, PadIfNeeded, RandomCrop, ColorJitter, HorizontalFlip, Normalize) and
the label remap of datasets/cityscapes.py:150-156.  At 1024 x 2048 a CPU pipeline costs tens
of milliseconds per image, which starves a GPU that trains at hundreds of images per second.

Split of work:

* host (DataLoader worker): decode the PNGs and draw the per-sample random parameters with
  :func:`draw_params`, which walks the SAME ``transforms.Compose`` and consumes the SAME
  ``numpy.random.Generator`` draws, in the same order, as the CPU path -- both paths see one
  augmentation stream per (seed, epoch, index);
* device: :func:`augment_batch` turns the raw uint8 batch into the normalised crop batch and
  the remapped label batch in one kernel pass (plus a per-image grey-level reduction when a
  sample's jitter has a contrast op).

Resampling follows albumentations / OpenCV rather than the CPU path's PIL: bilinear with
half-pixel centres rounded to uint8 (cv2.INTER_LINEAR, no antialiasing) and masks nearest
with ``floor(y * scale)`` (cv2.INTER_NEAREST); ``Scale`` and ``RandomScale`` compose into one
resample of the source (one interpolation instead of two).  Colour jitter, pad values,
re-quantisation and normalisation match ``datasets/transforms.py`` exactly.
:func:`augment_reference` is the PyTorch formulation (CPU path and numerics oracle).
"""
from __future__ import annotations

import numpy as np
import torch

from ._ext import ops, use_hip

# parameter row layout (= AugParam in csrc/include/rtseg_launch.h)
NH, NW, TOP, LEFT, CY, CX, FLIP, NOPS, CODE, BRIGHT, CONTRAST, SAT, HUE = range(13)
NPARAMS = 13
OP_BRIGHT, OP_CONTRAST, OP_SAT, OP_HUE = range(4)


class AugmentSpec:
    """Static part of a training pipeline: crop size, pad values, normalisation."""

    def __init__(self, crop_h, crop_w, mean, std, pad_value=114, mask_pad=0):
        self.crop_h, self.crop_w = int(crop_h), int(crop_w)
        self.mean = tuple(float(v) for v in mean)
        self.std = tuple(float(v) for v in std)
        self.pad_value, self.mask_pad = float(pad_value), int(mask_pad)


def draw_params(transform, src_h: int, src_w: int, rng: np.random.Generator):
    """Walk a ``transforms.Compose`` and draw one sample's parameters.

    Returns ``(params float32[NPARAMS], AugmentSpec)``.  Every random draw is made by the same
    transform attribute, in the same order, as ``transform(image, mask, rng)`` would make it.
    """
    from ..datasets import transforms as T

    h, w = int(src_h), int(src_w)
    top = left = 0
    canvas_h, canvas_w = h, w
    crop = None
    p = np.zeros(NPARAMS, np.float32)
    p[BRIGHT] = p[CONTRAST] = p[SAT] = 1.0
    pad_value, mask_pad = 114, 0
    mean, std = (0.0, 0.0, 0.0), (1.0, 1.0, 1.0)
    normalized = False
    for t in transform.transforms:
        if isinstance(t, T.Scale):
            if t.scale != 1.0:
                h, w = int(h * t.scale), int(w * t.scale)
                canvas_h, canvas_w = h, w
        elif isinstance(t, T.RandomScale):
            if not (t.range[0] == t.range[1] == 1.0):
                s = rng.uniform(*t.range)
                h, w = max(1, int(round(h * s))), max(1, int(round(w * s)))
                canvas_h, canvas_w = h, w
        elif isinstance(t, T.PadIfNeeded):
            ph, pw = max(0, t.mh - h), max(0, t.mw - w)
            top, left = ph // 2, pw // 2
            canvas_h, canvas_w = h + ph, w + pw
            pad_value, mask_pad = t.value, t.mask_value
        elif isinstance(t, T.RandomCrop):
            if canvas_h < t.h or canvas_w < t.w:
                raise ValueError(f"RandomCrop {t.h}x{t.w} larger than the {canvas_h}x{canvas_w} canvas")
            p[CY] = int(rng.integers(0, canvas_h - t.h + 1))
            p[CX] = int(rng.integers(0, canvas_w - t.w + 1))
            crop = (t.h, t.w)
        elif isinstance(t, T.ColorJitter):
            if rng.random() < t.p:
                ops_ = []
                if t.b:
                    p[BRIGHT] = t._factor(rng, t.b)
                    ops_.append(OP_BRIGHT)
                if t.c:
                    p[CONTRAST] = t._factor(rng, t.c)
                    ops_.append(OP_CONTRAST)
                if t.s:
                    p[SAT] = t._factor(rng, t.s)
                    ops_.append(OP_SAT)
                if t.hue:
                    p[HUE] = rng.uniform(-t.hue, t.hue)
                    ops_.append(OP_HUE)
                code = 0
                for k, j in enumerate(rng.permutation(len(ops_))):
                    code |= ops_[int(j)] << (2 * k)
                p[NOPS], p[CODE] = len(ops_), code
        elif isinstance(t, T.HorizontalFlip):
            if t.p > 0 and rng.random() < t.p:
                p[FLIP] = 1
        elif isinstance(t, T.Normalize):
            mean, std = tuple(t.mean.tolist()), tuple(t.std.tolist())
            normalized = True
        else:
            raise NotImplementedError(f"GPU augmentation does not support {type(t).__name__}")
    if not normalized:
        raise ValueError("the pipeline must end with Normalize")
    p[NH], p[NW], p[TOP], p[LEFT] = h, w, top, left
    if crop is None:
        crop = (canvas_h, canvas_w)
    return p, AugmentSpec(crop[0], crop[1], mean, std, pad_value, mask_pad)


def has_contrast(params: torch.Tensor) -> bool:
    """Whether any row's jitter sequence contains a contrast op (host-side check)."""
    p = params.detach().cpu()
    codes, nops = p[:, CODE].to(torch.int64), p[:, NOPS].to(torch.int64)
    for c, n in zip(codes.tolist(), nops.tolist()):
        if any(((c >> (2 * k)) & 3) == OP_CONTRAST for k in range(n)):
            return True
    return False


# ----------------------------------------------------------------------------- reference
def _lin_index(out_n, in_n, device):
    scale = in_n / out_n
    src = ((torch.arange(out_n, device=device, dtype=torch.float32) + 0.5) * scale - 0.5).clamp_min(0)
    i0 = src.to(torch.int64).clamp_max(in_n - 1)
    i1 = torch.where(i0 < in_n - 1, i0 + 1, i0)
    return i0, i1, src - i0.to(torch.float32)


def _rgb_to_hsv(x):
    r, g, b = x[..., 0], x[..., 1], x[..., 2]
    mx, mn = x.max(-1).values, x.min(-1).values
    d = mx - mn
    nz = d > 1e-12
    dd = torch.where(nz, d, torch.ones_like(d))
    rc, gc, bc = (mx - r) / dd, (mx - g) / dd, (mx - b) / dd
    h = torch.where(r == mx, bc - gc, torch.where(g == mx, 2.0 + rc - bc, 4.0 + gc - rc))
    h = h / 6.0
    h = torch.where(nz, h - torch.floor(h), torch.zeros_like(h))
    s = torch.where(mx > 1e-12, d / torch.where(mx > 1e-12, mx, torch.ones_like(mx)), torch.zeros_like(mx))
    return h, s, mx


def _hsv_to_rgb(h, s, v):
    i = torch.floor(h * 6.0)
    f = h * 6.0 - i
    p, q, t = v * (1 - s), v * (1 - s * f), v * (1 - s * (1 - f))
    i = i.to(torch.int64) % 6
    r = torch.stack([v, q, p, p, t, v], -1).gather(-1, i[..., None])[..., 0]
    g = torch.stack([t, v, v, q, p, p], -1).gather(-1, i[..., None])[..., 0]
    b = torch.stack([p, p, t, v, v, q], -1).gather(-1, i[..., None])[..., 0]
    return torch.stack([r, g, b], -1)


_GREY = (0.299, 0.587, 0.114)


def _grey(x):
    return x[..., 0] * _GREY[0] + x[..., 1] * _GREY[1] + x[..., 2] * _GREY[2]


def _jitter(op, p, x, cmean):
    if op == OP_BRIGHT:
        return (x * float(p[BRIGHT])).clamp(0, 1)
    if op == OP_CONTRAST:
        return ((x - cmean) * float(p[CONTRAST]) + cmean).clamp(0, 1)
    if op == OP_SAT:
        g = _grey(x)[..., None]
        return (g + (x - g) * float(p[SAT])).clamp(0, 1)
    h, s, v = _rgb_to_hsv(x)
    h = h + float(p[HUE])
    return _hsv_to_rgb(h - torch.floor(h), s, v)


def augment_reference(img, msk, params, lut, spec: AugmentSpec, out_dtype=torch.float32, mask_dtype=torch.int64):
    """PyTorch formulation of the kernel.  img uint8 [N, H, W, 3], msk uint8 [N, H, W] or None,
    params fp32 [N, NPARAMS], lut uint8 [256].  Returns (images [N, 3, ch, cw], masks [N, ch, cw])."""
    n, H, W, _ = img.shape
    ch, cw = spec.crop_h, spec.crop_w
    dev = img.device
    outs, mouts = [], []
    prm = params.detach().cpu().numpy()
    lut_t = lut.to(dev, torch.int64)
    for b in range(n):
        p = prm[b]
        nh, nw = int(p[NH]), int(p[NW])
        oy = torch.arange(ch, device=dev)
        ox = torch.arange(cw, device=dev)
        xx = (cw - 1 - ox) if p[FLIP] else ox
        py = oy + int(p[CY]) - int(p[TOP])
        px = xx + int(p[CX]) - int(p[LEFT])
        vy = (py >= 0) & (py < nh)
        vx = (px >= 0) & (px < nw)
        pyc, pxc = py.clamp(0, nh - 1), px.clamp(0, nw - 1)
        y0, y1, ly = _lin_index(nh, H, dev)
        x0, x1, lx = _lin_index(nw, W, dev)
        y0, y1, ly = y0[pyc], y1[pyc], ly[pyc][:, None, None]
        x0, x1, lx = x0[pxc], x1[pxc], lx[pxc][None, :, None]
        src = img[b].to(torch.float32)
        top = src[y0][:, x0] + lx * (src[y0][:, x1] - src[y0][:, x0])
        bot = src[y1][:, x0] + lx * (src[y1][:, x1] - src[y1][:, x0])
        rgb = torch.round(top + ly * (bot - top)).clamp(0, 255)
        valid = (vy[:, None] & vx[None, :])[..., None]
        rgb = torch.where(valid, rgb, torch.full_like(rgb, spec.pad_value))
        nops, code = int(p[NOPS]), int(p[CODE])
        if nops:
            x = rgb / 255.0
            seq = [(code >> (2 * k)) & 3 for k in range(nops)]
            cmean = 0.0
            if OP_CONTRAST in seq:
                pre = x
                for op in seq[: seq.index(OP_CONTRAST)]:
                    pre = _jitter(op, p, pre, 0.0)
                cmean = float(_grey(pre).to(torch.float64).mean())
            for op in seq:
                x = _jitter(op, p, x, cmean)
            rgb = torch.floor(x * 255.0 + 0.5).clamp(0, 255)
        mean = torch.tensor(spec.mean, device=dev, dtype=torch.float32)
        std = torch.tensor(spec.std, device=dev, dtype=torch.float32)
        outs.append(((rgb / 255.0 - mean) / std).permute(2, 0, 1))
        if msk is not None:
            sy, sx = H / nh, W / nw
            my = torch.floor(pyc.to(torch.float32) * sy).to(torch.int64).clamp_max(H - 1)
            mx = torch.floor(pxc.to(torch.float32) * sx).to(torch.int64).clamp_max(W - 1)
            raw = msk[b].to(torch.int64)[my][:, mx]
            raw = torch.where(valid[..., 0], raw, torch.full_like(raw, spec.mask_pad))
            mouts.append(lut_t[raw])
    images = torch.stack(outs).to(out_dtype)
    masks = torch.stack(mouts).to(mask_dtype) if msk is not None else None
    return images, masks


# ----------------------------------------------------------------------------- public op
def augment_batch(img, msk, params, lut, spec: AugmentSpec, out_dtype=torch.float32, channels_last=False,
                  mask_dtype=torch.int64):
    """Raw uint8 batch -> (normalised [N, 3, ch, cw] images, remapped [N, ch, cw] labels).

    GPU tensors run the HIP kernel (one pass; a grey-level reduction first if a sample's jitter
    has a contrast op); CPU tensors run :func:`augment_reference`."""
    if not use_hip(img):
        return augment_reference(img, msk, params, lut, spec, out_dtype, mask_dtype)
    dev = img.device
    n = img.shape[0]
    fmt = torch.channels_last if channels_last else torch.contiguous_format
    out = torch.empty(n, 3, spec.crop_h, spec.crop_w, device=dev, dtype=out_dtype, memory_format=fmt)
    mout = torch.empty(n, spec.crop_h, spec.crop_w, device=dev, dtype=mask_dtype) if msk is not None else None
    norm = torch.tensor(spec.mean + spec.std, dtype=torch.float32).to(dev, non_blocking=True)
    params_d = params.to(dev, torch.float32, non_blocking=True).contiguous()
    ops().augment(img.contiguous(), None if msk is None else msk.contiguous(), params_d,
                  lut.to(dev, torch.uint8).contiguous(), norm, out, mout, spec.pad_value, spec.mask_pad,
                  has_contrast(params))
    return out, mout


__all__ = ["AugmentSpec", "draw_params", "augment_batch", "augment_reference", "has_contrast", "NPARAMS"]
