"""Dilated grouped convolutions through space-to-batch.

Reference: RegSeg's ``DBlock`` (reference models/regseg.py:62-127) -- grouped 3x3 convs (group
width 16) with dilation up to 14.  PyTorch never hands a conv that is both grouped and dilated
to MIOpen; it falls back to im2col + one GEMM per group per image (``profiles/r1_regseg_infer``:
~13k tiny launches per run, RegSeg the slowest model of the zoo relative to the reference).

A stride-1 'same' conv with dilation (dh, dw) only ever combines pixels of one residue class
(h mod dh, w mod dw), so it is exactly the dilation-1 conv applied to each of the dh*dw
sub-grids.  :class:`DilatedGroupConv2d` therefore rearranges x [N, C, H, W] (zero-padded up to
multiples of the dilation; zeros there are what the original padding reads) into
[N*dh*dw, C, H/dh, W/dw], runs the grouped dilation-1 conv on MIOpen (CK grouped-conv
kernels), and rearranges back -- two bandwidth-bound copies instead of the im2col fallback.
:func:`convert_dilated_group_convs` swaps the class of every eligible ``nn.Conv2d`` (parameters
and checkpoint keys unchanged); CPU tensors keep ``F.conv2d``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def dilated_group_ok(conv: nn.Module) -> bool:
    if type(conv) is not nn.Conv2d or conv.groups == 1 or conv.groups == conv.in_channels:
        return False  # dense convs reach MIOpen already; depth-wise ones run on dwconv.hip
    if conv.padding_mode != "zeros" or isinstance(conv.padding, str) or tuple(conv.stride) != (1, 1):
        return False
    if max(conv.dilation) < 2:
        return False
    return all(k % 2 == 1 and p == d * (k - 1) // 2
               for k, p, d in zip(conv.kernel_size, conv.padding, conv.dilation))


def dilated_group_conv2d(x, weight, bias, dilation, groups):
    """Space-to-batch dilated grouped conv.  Both rearrangements are done on the channels-last
    (NHWC) view, so each side is ONE copy (plus one for the crop when H or W is not a
    multiple of the dilation)."""
    n, c, h, w = x.shape
    dh, dw = dilation
    hp, wp = -(-h // dh) * dh, -(-w // dw) * dw
    xn = x.permute(0, 2, 3, 1)  # NHWC view (free for a channels-last x)
    if (hp, wp) != (h, w):
        xn = F.pad(xn, (0, 0, 0, wp - w, 0, hp - h))
    hs, ws = hp // dh, wp // dw
    xs = xn.reshape(n, hs, dh, ws, dw, c).permute(0, 2, 4, 1, 3, 5).reshape(n * dh * dw, hs, ws, c)
    xs = xs.permute(0, 3, 1, 2)  # NCHW logical, channels-last physical
    kh, kw = weight.shape[2:]
    ys = F.conv2d(xs, weight, bias, 1, ((kh - 1) // 2, (kw - 1) // 2), 1, groups)
    co = ys.shape[1]
    yn = ys.permute(0, 2, 3, 1).reshape(n, dh, dw, hs, ws, co).permute(0, 3, 1, 4, 2, 5).reshape(n, hp, wp, co)
    y = yn.permute(0, 3, 1, 2)
    if (hp, wp) != (h, w):
        y = y[:, :, :h, :w].contiguous(memory_format=torch.channels_last)
    return y


class DilatedGroupConv2d(nn.Conv2d):
    """``nn.Conv2d`` (grouped + dilated) run as space-to-batch on the GPU (module docstring)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from ._ext import use_hip

        if not x.is_cuda or not use_hip(x):  # RTSEG_DISABLE_HIP=1: the stock conv, for A/B runs
            return super().forward(x)
        return dilated_group_conv2d(x, self.weight, self.bias, tuple(self.dilation), self.groups)


def convert_dilated_group_convs(model: nn.Module) -> nn.Module:
    for m in model.modules():
        if dilated_group_ok(m):
            m.__class__ = DilatedGroupConv2d
    return model
