"""PixelShuffle / PixelUnshuffle / channel shuffle on the HIP remap kernel (``shuffle.hip``).

Reference: models/farseenet.py:59,82 (``nn.PixelShuffle`` sub-pixel fusion) and
models/modules.py:18-32 (``channel_shuffle``: LEDNet, Lite-HRNet).  PyTorch implements these as
reshape + permute + copy, which for channels-last activations first materialises an NCHW copy;
here each is one gather pass that keeps the input's memory format.  Backward = the inverse remap.
CPU tensors run the PyTorch formulation.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import ops, use_hip

PIXEL, PIXEL_INV, CHANNEL = 0, 1, 2


def _inverse(mode, r, c):
    if mode == PIXEL:
        return PIXEL_INV, r
    if mode == PIXEL_INV:
        return PIXEL, r
    return CHANNEL, c // r


class _ShuffleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mode, r):
        ctx.inv = _inverse(mode, r, x.shape[1])
        return ops().shuffle(x, mode, r)

    @staticmethod
    def backward(ctx, g):
        return _ShuffleFn.apply(g, *ctx.inv), None, None


def _ok(x):
    return (x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16, torch.float16) and x.numel() < 2 ** 32
            and use_hip(x, "shuffle"))


def pixel_shuffle(x: torch.Tensor, r: int) -> torch.Tensor:
    if x.is_cuda and _ok(x) and r > 1:
        return _ShuffleFn.apply(x, PIXEL, int(r))
    return F.pixel_shuffle(x, r)


def pixel_unshuffle(x: torch.Tensor, r: int) -> torch.Tensor:
    if x.is_cuda and _ok(x) and r > 1:
        return _ShuffleFn.apply(x, PIXEL_INV, int(r))
    return F.pixel_unshuffle(x, r)


def channel_shuffle(x: torch.Tensor, groups: int = 2) -> torch.Tensor:
    """ShuffleNet channel shuffle: [N, g*k, H, W] -> interleave the g groups."""
    if x.is_cuda and _ok(x) and 1 < groups < x.shape[1]:
        return _ShuffleFn.apply(x, CHANNEL, int(groups))
    n, c, h, w = x.shape
    return x.reshape(n, groups, c // groups, h, w).transpose(1, 2).reshape(n, c, h, w)


class PixelShuffle(nn.PixelShuffle):
    def forward(self, x):
        return pixel_shuffle(x, self.upscale_factor)


class PixelUnshuffle(nn.PixelUnshuffle):
    def forward(self, x):
        return pixel_unshuffle(x, self.downscale_factor)


def convert_pixel_shuffle(model: nn.Module) -> nn.Module:
    """Swap nn.PixelShuffle / nn.PixelUnshuffle modules onto the HIP remap (in place)."""
    for m in model.modules():
        if type(m) is nn.PixelShuffle:
            m.__class__ = PixelShuffle
        elif type(m) is nn.PixelUnshuffle:
            m.__class__ = PixelUnshuffle
    return model


__all__ = ["pixel_shuffle", "pixel_unshuffle", "channel_shuffle", "PixelShuffle", "PixelUnshuffle",
           "convert_pixel_shuffle"]
