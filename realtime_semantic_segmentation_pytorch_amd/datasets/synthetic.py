"""Synthetic Cityscapes-shaped data.

* :class:`SyntheticSegDataset` -- a map-style CPU dataset (deterministic per
  index) for the CPU plumbing config and loader tests.
* :class:`DeviceBatches` -- device-resident random batches for benchmarks: a
  small pool of ``[N,3,H,W]`` images / ``[N,H,W]`` int64 masks generated ONCE on
  the GPU and cycled, so the input pipeline costs nothing inside a timed step
  (the benchmark measures the training step, as BASELINE.json specifies
  synthetic 1024x2048 19-class data).
"""
from __future__ import annotations

import torch
from torch.utils.data import Dataset


def _masks_like(gen, n, h, w, num_class, ignore_index, device):
    """Blocky label maps (8x8 cells) with ~5% ignore pixels -- closer to real
    segmentation statistics than i.i.d. noise and identical on every backend."""
    ch, cw = max(1, (h + 7) // 8), max(1, (w + 7) // 8)
    cells = torch.randint(0, num_class, (n, 1, ch, cw), generator=gen, device="cpu").float()
    m = torch.nn.functional.interpolate(cells, size=(h, w), mode="nearest").long().squeeze(1)
    ign = torch.rand((n, h, w), generator=gen) < 0.05
    m[ign] = ignore_index
    return m.to(device)


def class_palette(num_class: int) -> torch.Tensor:
    """[num_class, 3] well-separated colours (normalised-image units) for the learnable task: the
    points of a {-1, 0, 1}^3 grid (up to 27 classes: any two differ by >= 1 in some channel), a
    4-level grid (>= 2/3) up to 64 classes."""
    levels = 3 if num_class <= 27 else 4 if num_class <= 64 else 1 + int(round(num_class ** (1 / 3) + 0.5))
    vals = torch.linspace(-1.0, 1.0, levels)
    grid = torch.cartesian_prod(vals, vals, vals)
    return grid[:num_class].clone()


def learnable_sample(gen, h, w, num_class, ignore_index, cell=32, noise=0.15, ignore_frac=0.02):
    """One (image [3, H, W], label [H, W]) pair whose label is a function of the image: a map of
    ``cell`` x ``cell`` blocks of random classes, each block painted in its class colour
    (:func:`class_palette`) plus Gaussian noise; ``ignore_frac`` of the pixels are ignore-labelled
    (their colour still follows the block's class)."""
    ch, cw = max(1, (h + cell - 1) // cell), max(1, (w + cell - 1) // cell)
    cells = torch.randint(0, num_class, (1, 1, ch, cw), generator=gen).float()
    lbl = torch.nn.functional.interpolate(cells, size=(ch * cell, cw * cell), mode="nearest")[0, 0, :h, :w].long()
    img = class_palette(num_class)[lbl].permute(2, 0, 1).contiguous()
    img = img + noise * torch.randn((3, h, w), generator=gen)
    ign = torch.rand((h, w), generator=gen) < ignore_frac
    lbl[ign] = ignore_index
    return img, lbl


class SyntheticSegDataset(Dataset):
    """``learnable=False``: random images with blocky labels uncorrelated with them (throughput,
    plumbing); ``learnable=True``: :func:`learnable_sample` -- colour-coded blocks, so training
    must raise validation mIoU (convergence tests, ``config.synthetic_learnable``)."""

    def __init__(self, length=2, size=(64, 128), num_class=19, ignore_index=255, seed=0, learnable=False,
                 cell=32):
        self.length, self.size, self.num_class = length, tuple(size), num_class
        self.ignore_index, self.seed = ignore_index, seed
        self.learnable, self.cell = bool(learnable), int(cell)

    def __len__(self):
        return self.length

    def __getitem__(self, key):
        index = int(key[0]) if isinstance(key, (tuple, list)) else int(key)
        g = torch.Generator().manual_seed(self.seed * 100003 + index)
        h, w = self.size
        if self.learnable:
            return learnable_sample(g, h, w, self.num_class, self.ignore_index, self.cell)
        img = torch.randn((3, h, w), generator=g)
        mask = _masks_like(g, 1, h, w, self.num_class, self.ignore_index, "cpu")[0]
        return img, mask


class DeviceBatches:
    """Cycle over ``pool`` pre-generated device batches."""

    def __init__(self, batch_size, size, num_class=19, ignore_index=255, device="cuda", pool=2,
                 dtype=torch.float32, channels_last=False, seed=0, length=None):
        g = torch.Generator().manual_seed(seed)
        h, w = size
        self.batches = []
        for _ in range(pool):
            img = torch.randn((batch_size, 3, h, w), generator=g).to(device=device, dtype=dtype)
            if channels_last:
                img = img.contiguous(memory_format=torch.channels_last)
            mask = _masks_like(g, batch_size, h, w, num_class, ignore_index, device)
            self.batches.append((img, mask))
        self.length = length
        self._i = 0

    def __len__(self):
        return self.length if self.length is not None else len(self.batches)

    def next(self):
        b = self.batches[self._i % len(self.batches)]
        self._i += 1
        return b

    def __iter__(self):
        for i in range(len(self)):
            yield self.batches[i % len(self.batches)]
