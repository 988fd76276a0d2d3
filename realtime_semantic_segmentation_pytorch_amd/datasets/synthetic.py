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


class SyntheticSegDataset(Dataset):
    def __init__(self, length=2, size=(64, 128), num_class=19, ignore_index=255, seed=0):
        self.length, self.size, self.num_class = length, tuple(size), num_class
        self.ignore_index, self.seed = ignore_index, seed

    def __len__(self):
        return self.length

    def __getitem__(self, key):
        index = int(key[0]) if isinstance(key, (tuple, list)) else int(key)
        g = torch.Generator().manual_seed(self.seed * 100003 + index)
        h, w = self.size
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
