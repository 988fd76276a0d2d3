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

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

# ---------------------------------------------------------------------------------------------
# Dead-tap pruning.
#
# A conv whose reach exceeds the feature map -- dilation >= the map extent (LEDNet's dilation-17
# (3, 1) convs on a 16-row map, LiteSeg's dilation-12/18 branches and RegSeg's dilation-14
# DBlocks at 1/16 scale, SMP ASPP rates 12/24/36) -- has taps that read nothing but zero
# padding for EVERY output pixel.  Dropping them is exact: the output is unchanged and the
# dropped weights' gradient is exactly 0.  It removes work (a 3x3 conv on a map shorter than its
# dilation is a 1x3 conv) and it keeps such geometries away from MIOpen: MIOpen's NHWC solvers
# have faulted the GPU on exactly these (round-1 find-mode search on LEDNet / CFPNet shapes, and
# the intermittent round-2/3 fault in the single-process zoo checks, always on LEDNet, LiteSeg or
# RegSeg backward in fp32, where every dense conv is MIOpen's).
# ---------------------------------------------------------------------------------------------


def _fmt(x: torch.Tensor):
    cl = x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous()
    return torch.channels_last if cl else torch.contiguous_format


def _out_len(extent: int, k: int, s: int, p: int, d: int) -> int:
    return (extent + 2 * p - d * (k - 1) - 1) // s + 1


def live_taps(extent: int, k: int, s: int, p: int, d: int):
    """``(lo, hi)``: the taps along one axis that read an in-range input for at least one output
    position (a contiguous range), or None when no tap ever does."""
    out = _out_len(extent, k, s, p, d)
    if out <= 0:
        return None
    lo, hi = 0, k - 1
    while lo <= hi and lo * d - p + (out - 1) * s < 0:  # tap only ever reads the left padding
        lo += 1
    while hi >= lo and hi * d - p >= extent:  # ... or only the right padding
        hi -= 1
    return (lo, hi) if lo <= hi else None


def has_dead_taps(hw, kernel_size, stride, padding, dilation) -> bool:
    """Whether a zero-padded conv over an ``hw`` map has taps that never read the map (cheap:
    only the first and last tap of each axis can be dead first)."""
    for e, k, s, p, d in zip(hw, kernel_size, stride, padding, dilation):
        if k > 1 and (p > (_out_len(e, k, s, p, d) - 1) * s or (k - 1) * d - p >= e):
            return True
    return False


def pruned_conv2d(x, weight, bias, stride, padding, dilation, groups):
    """``F.conv2d`` with the dead taps of ``weight`` removed (exact; see above).  Padding that
    becomes asymmetric is applied (or cropped) explicitly."""
    stride, padding, dilation = tuple(stride), tuple(padding), tuple(dilation)
    hw = tuple(x.shape[2:])
    if not has_dead_taps(hw, weight.shape[2:], stride, padding, dilation):
        return F.conv2d(x, weight, bias, stride, padding, dilation, groups)
    spans = [live_taps(e, k, s, p, d)
             for e, k, s, p, d in zip(hw, weight.shape[2:], stride, padding, dilation)]
    if None in spans:  # an all-padding conv: nothing to keep, leave it as is
        return F.conv2d(x, weight, bias, stride, padding, dilation, groups)
    w = weight[:, :, spans[0][0]:spans[0][1] + 1, spans[1][0]:spans[1][1] + 1]
    w = w.contiguous(memory_format=_fmt(x))
    lr, dil = [], []
    for (lo, hi), e, k, s, p, d in zip(spans, hw, weight.shape[2:], stride, padding, dilation):
        kk = hi - lo + 1
        dd = d if kk > 1 else 1
        left = p - lo * d
        right = (_out_len(e, k, s, p, d) - 1) * s + dd * (kk - 1) + 1 - e - left
        lr.append((left, right))
        dil.append(dd)
    if all(a == b >= 0 for a, b in lr):
        return F.conv2d(x, w, bias, stride, (lr[0][0], lr[1][0]), tuple(dil), groups)
    xp = F.pad(x, (lr[1][0], lr[1][1], lr[0][0], lr[0][1]))
    return F.conv2d(xp, w, bias, stride, 0, tuple(dil), groups)


class PrunedConv2d(nn.Conv2d):
    """``nn.Conv2d`` whose forward drops dead taps for the current input size
    (:func:`pruned_conv2d`, on every device: exact); identical to ``nn.Conv2d`` whenever no tap
    is dead."""

    def _conv_forward(self, input, weight, bias):
        if (bias is not None and input.is_cuda and input.dim() == 4 and self.groups == 1
                and os.environ.get("RTSEG_BIAS_ADD", "1") != "0"):
            # bias-free conv + bias_add: the bias gradient on the HIP channel-sum pass
            from .bn import bias_add

            return bias_add(self._conv_forward(input, weight, None), bias)
        if (self.padding_mode != "zeros" or input.dim() != 4
                or not has_dead_taps(input.shape[2:], self.kernel_size, self.stride, self.padding, self.dilation)):
            return super()._conv_forward(input, weight, bias)
        return pruned_conv2d(input, weight, bias, self.stride, self.padding, self.dilation, self.groups)


def prunable(conv: nn.Module) -> bool:
    """Spatial convs (dead taps) and biased dense ones (their bias goes through ``bias_add``)."""
    return (type(conv) is nn.Conv2d and conv.padding_mode == "zeros" and not isinstance(conv.padding, str)
            and (max(conv.kernel_size) > 1 or (conv.bias is not None and conv.groups == 1)))


def convert_pruned_convs(model: nn.Module) -> nn.Module:
    """Swap every remaining plain ``nn.Conv2d`` with a spatial kernel to :class:`PrunedConv2d`
    (run after the other converters; parameters and checkpoint keys unchanged)."""
    for m in model.modules():
        if prunable(m):
            m.__class__ = PrunedConv2d
    return model


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
    ys = pruned_conv2d(xs, weight, bias, (1, 1), ((kh - 1) // 2, (kw - 1) // 2), (1, 1), groups)
    co = ys.shape[1]
    yn = ys.permute(0, 2, 3, 1).reshape(n, dh, dw, hs, ws, co).permute(0, 3, 1, 4, 2, 5).reshape(n, hp, wp, co)
    y = yn.permute(0, 3, 1, 2)
    if (hp, wp) != (h, w):
        y = y[:, :, :h, :w].contiguous(memory_format=torch.channels_last)
    return y


def dilated_group_pruned(x, weight, bias, dilation, groups):
    """:func:`dilated_group_conv2d` after dropping dead taps: a dilation >= the map extent
    leaves only the centre tap on that axis, which then needs no space-to-batch along it (what
    stays is still 'same' and symmetric)."""
    w, dil = weight, list(dilation)
    for a, (e, k, d) in enumerate(zip(x.shape[2:], weight.shape[2:], dilation)):
        c = (k - 1) // 2
        m = min(c, -(-e // d) - 1)
        if m < c:
            w = w.narrow(2 + a, c - m, 2 * m + 1)
            dil[a] = d if m > 0 else 1
    if max(dil) < 2:
        kh, kw = w.shape[2:]
        return F.conv2d(x, w.contiguous(memory_format=_fmt(x)), bias, 1,
                        ((kh - 1) // 2, (kw - 1) // 2), 1, groups)
    return dilated_group_conv2d(x, w, bias, tuple(dil), groups)


class DilatedGroupConv2d(nn.Conv2d):
    """``nn.Conv2d`` (grouped + dilated) run as space-to-batch on the GPU (module docstring)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from ._ext import use_hip

        if not x.is_cuda or not use_hip(x, "dilated"):
            # CPU / RTSEG_DISABLE_HIP=1 (the stock yardstick): the stock conv, dead taps dropped --
            # no fallback hands a padding-only tap to the vendor library (profiles/r5_fault)
            return pruned_conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups)
        from .conv import grouped_as_dense, grouped_dense_ok

        if grouped_dense_ok(x, self):  # training: the block-diagonal dense route (ops/conv.py)
            return grouped_as_dense(x, self)
        return dilated_group_pruned(x, self.weight, self.bias, tuple(self.dilation), self.groups)


def convert_dilated_group_convs(model: nn.Module) -> nn.Module:
    for m in model.modules():
        if dilated_group_ok(m):
            m.__class__ = DilatedGroupConv2d
    return model
