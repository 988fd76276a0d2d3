"""Augmentation pipeline (replaces albumentations, absent in this environment).

Semantics follow the reference pipeline (datasets/cityscapes.py:115-131 and
utils/transforms.py:12-68) as implemented by albumentations:

* ``Scale(s)``           -- resize by a factor (bilinear image / nearest mask)
* ``RandomScale(lim)``   -- factor ~ U(1+lim[0], 1+lim[1]) (scalar lim -> +-lim)
* ``PadIfNeeded``        -- centred constant pad to >= (h, w): image 114, mask 0
* ``RandomCrop``         -- uniform crop
* ``ColorJitter``        -- p=0.5; brightness/contrast/saturation factors ~
                            U(max(0,1-v), 1+v), hue shift ~ U(-0.2, 0.2), random order
* ``HorizontalFlip(p)``
* ``Normalize(mean,std)``-- on [0,1]-scaled pixels
* ``ResizeToSquare(n)``  -- zero-pad to square then resize (the mask IS padded
                            here; the reference forgets to -- SURVEY A.1 #17)

Every transform maps ``(image HxWx3 uint8|float32, mask HxW | None)`` to the
same pair and draws randomness from a caller-provided ``numpy.random.Generator``.
"""
from __future__ import annotations

import numpy as np
from PIL import Image

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _resize(img: np.ndarray, h: int, w: int, nearest: bool) -> np.ndarray:
    if img.shape[0] == h and img.shape[1] == w:
        return img
    mode = Image.NEAREST if nearest else Image.BILINEAR
    if img.dtype == np.uint8:
        return np.asarray(Image.fromarray(img).resize((w, h), mode))
    chans = [np.asarray(Image.fromarray(img[..., c].astype(np.float32), mode="F").resize((w, h), mode))
             for c in range(img.shape[2])] if img.ndim == 3 else None
    if chans is None:
        return np.asarray(Image.fromarray(img.astype(np.float32), mode="F").resize((w, h), mode))
    return np.stack(chans, axis=-1)


class Compose:
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, image, mask=None, rng=None):
        rng = rng if rng is not None else np.random.default_rng()
        for t in self.transforms:
            image, mask = t(image, mask, rng)
        return image, mask


class Scale:
    def __init__(self, scale=1.0):
        self.scale = float(scale)

    def __call__(self, image, mask, rng):
        if self.scale == 1.0:
            return image, mask
        h, w = image.shape[:2]
        nh, nw = int(h * self.scale), int(w * self.scale)
        return _resize(image, nh, nw, False), (None if mask is None else _resize(mask, nh, nw, True))


class RandomScale:
    def __init__(self, scale_limit=0.0):
        if isinstance(scale_limit, (list, tuple)):
            lo, hi = float(scale_limit[0]), float(scale_limit[-1])
        else:
            lo, hi = -float(scale_limit), float(scale_limit)
        self.range = (1.0 + lo, 1.0 + hi)

    def __call__(self, image, mask, rng):
        if self.range[0] == self.range[1] == 1.0:
            return image, mask
        s = rng.uniform(*self.range)
        h, w = image.shape[:2]
        nh, nw = max(1, int(round(h * s))), max(1, int(round(w * s)))
        return _resize(image, nh, nw, False), (None if mask is None else _resize(mask, nh, nw, True))


class PadIfNeeded:
    def __init__(self, min_height, min_width, value=114, mask_value=0):
        self.mh, self.mw = int(min_height), int(min_width)
        self.value, self.mask_value = value, mask_value

    def __call__(self, image, mask, rng):
        h, w = image.shape[:2]
        ph, pw = max(0, self.mh - h), max(0, self.mw - w)
        if ph == 0 and pw == 0:
            return image, mask
        top, left = ph // 2, pw // 2
        pads = ((top, ph - top), (left, pw - left))
        image = np.pad(image, pads + ((0, 0),), mode="constant", constant_values=self.value)
        if mask is not None:
            mask = np.pad(mask, pads, mode="constant", constant_values=self.mask_value)
        return image, mask


class RandomCrop:
    def __init__(self, height, width):
        self.h, self.w = int(height), int(width)

    def __call__(self, image, mask, rng):
        h, w = image.shape[:2]
        y = int(rng.integers(0, h - self.h + 1))
        x = int(rng.integers(0, w - self.w + 1))
        image = image[y:y + self.h, x:x + self.w]
        if mask is not None:
            mask = mask[y:y + self.h, x:x + self.w]
        return image, mask


def _rgb_to_hsv(x):
    r, g, b = x[..., 0], x[..., 1], x[..., 2]
    mx = x.max(-1)
    mn = x.min(-1)
    d = mx - mn
    h = np.zeros_like(mx)
    nz = d > 1e-12
    rc = np.where(nz, (mx - r) / np.where(nz, d, 1), 0)
    gc = np.where(nz, (mx - g) / np.where(nz, d, 1), 0)
    bc = np.where(nz, (mx - b) / np.where(nz, d, 1), 0)
    h = np.where(r == mx, bc - gc, np.where(g == mx, 2.0 + rc - bc, 4.0 + gc - rc))
    h = np.where(nz, (h / 6.0) % 1.0, 0.0)
    s = np.where(mx > 1e-12, d / np.where(mx > 1e-12, mx, 1), 0)
    return h, s, mx


def _hsv_to_rgb(h, s, v):
    i = np.floor(h * 6.0)
    f = h * 6.0 - i
    p, q, t = v * (1 - s), v * (1 - s * f), v * (1 - s * (1 - f))
    i = i.astype(np.int32) % 6
    r = np.choose(i, [v, q, p, p, t, v])
    g = np.choose(i, [t, v, v, q, p, p])
    b = np.choose(i, [p, p, t, v, v, q])
    return np.stack([r, g, b], -1)


class ColorJitter:
    def __init__(self, brightness=0.0, contrast=0.0, saturation=0.0, hue=0.2, p=0.5):
        self.b, self.c, self.s, self.hue, self.p = brightness, contrast, saturation, hue, p

    @staticmethod
    def _factor(rng, v):
        return rng.uniform(max(0.0, 1 - v), 1 + v)

    def __call__(self, image, mask, rng):
        if rng.random() >= self.p:
            return image, mask
        x = image.astype(np.float32) / 255.0
        ops = []
        if self.b:
            f = self._factor(rng, self.b)
            ops.append(lambda z, f=f: np.clip(z * f, 0, 1))
        if self.c:
            f = self._factor(rng, self.c)
            ops.append(lambda z, f=f: np.clip((z - (z @ np.float32([0.299, 0.587, 0.114])).mean()) * f
                                              + (z @ np.float32([0.299, 0.587, 0.114])).mean(), 0, 1))
        if self.s:
            f = self._factor(rng, self.s)

            def sat(z, f=f):
                gray = (z @ np.float32([0.299, 0.587, 0.114]))[..., None]
                return np.clip(gray + (z - gray) * f, 0, 1)
            ops.append(sat)
        if self.hue:
            dh = rng.uniform(-self.hue, self.hue)

            def hue(z, dh=dh):
                h, s, v = _rgb_to_hsv(z)
                return _hsv_to_rgb((h + dh) % 1.0, s, v).astype(np.float32)
            ops.append(hue)
        for k in rng.permutation(len(ops)):
            x = ops[k](x)
        return (x * 255.0 + 0.5).clip(0, 255).astype(np.uint8), mask


class HorizontalFlip:
    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, image, mask, rng):
        if self.p > 0 and rng.random() < self.p:
            image = image[:, ::-1]
            if mask is not None:
                mask = mask[:, ::-1]
        return image, mask


class ResizeToSquare:
    def __init__(self, size):
        self.size = size

    def __call__(self, image, mask, rng):
        if self.size is None:
            return image, mask
        h, w = image.shape[:2]
        m = max(h, w)
        top, left = (m - h) // 2, (m - w) // 2
        pads = ((top, m - h - top), (left, m - w - left))
        image = np.pad(image, pads + ((0, 0),), mode="constant")
        if mask is not None:
            mask = np.pad(mask, pads, mode="constant")
        return (_resize(image, self.size, self.size, False),
                None if mask is None else _resize(mask, self.size, self.size, True))


class Normalize:
    def __init__(self, mean=IMAGENET_MEAN, std=IMAGENET_STD):
        self.mean = np.asarray(mean, np.float32)
        self.std = np.asarray(std, np.float32)

    def __call__(self, image, mask, rng):
        x = image.astype(np.float32) / 255.0
        return (x - self.mean) / self.std, mask


def to_tensor(image: np.ndarray):
    import torch

    return torch.from_numpy(np.ascontiguousarray(image.transpose(2, 0, 1)))


def train_transform(config, normalize=(IMAGENET_MEAN, IMAGENET_STD), square_size=None):
    ts = []
    if square_size is not None:
        ts.append(ResizeToSquare(square_size))
    ts += [
        Scale(config.scale),
        RandomScale(config.randscale),
        PadIfNeeded(config.crop_h, config.crop_w, 114, 0),
        RandomCrop(config.crop_h, config.crop_w),
        ColorJitter(config.brightness, config.contrast, config.saturation),
        HorizontalFlip(config.h_flip),
        Normalize(*normalize),
    ]
    return Compose(ts)


def val_transform(config, normalize=(IMAGENET_MEAN, IMAGENET_STD), square_size=None):
    ts = [ResizeToSquare(square_size)] if square_size is not None else []
    ts += [Scale(config.scale), Normalize(*normalize)]
    return Compose(ts)
