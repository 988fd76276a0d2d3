"""2-D pooling on the HIP kernels of ``csrc/kernels/pool.hip``.

Reference sites: DDRNet's DAPPM ``AvgPool2d(5/9/17)`` + global pool
(models/ddrnet.py:248-264), STDC's ``AvgPool2d(3, 2, 1)`` in every stride-2 module
(models/stdc.py:116), BiSeNetV2's stem ``MaxPool2d(3, 2, 1)``, GE ``AvgPool2d`` and
context-embedding global pool (models/bisenetv2.py:117,131,144), the PPM
``AdaptiveAvgPool2d(1/2/4/6)`` (models/modules.py:147) and the global pools of the
attention blocks and SMP decoders.

:func:`convert_pooling` swaps the class of every eligible pooling module to a
subclass whose forward takes the HIP path for GPU inputs (modules have no state,
so checkpoints are unaffected).  Semantics are ATen's: ``count_include_pad``
divisors, first-maximum argmax, adaptive windows ``[floor(o*I/O), ceil((o+1)*I/O))``.
``MaxPool2d(return_indices=True)`` returns PyTorch's int64 flat plane indices and
``MaxUnpool2d`` (kernel == stride, no padding: ENet / SegNet, reference enet.py:131,139 and
segnet.py:54,65) runs as a gather -- each output pixel reads its own window's index -- so
neither direction scatters or zero-fills.  Unsupported variants (``ceil_mode``,
``divisor_override``, dilation) keep the PyTorch module.  ``RTSEG_POOL=0`` disables the
path for A/B comparisons.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import ops, use_hip

_AVG, _MAX = 0, 1
_DTYPES = (torch.float32, torch.bfloat16, torch.float16)


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def _hip_ok(x: torch.Tensor) -> bool:
    return (x.dim() == 4 and x.dtype in _DTYPES and x.numel() < 2 ** 31 and use_hip(x, "pool")
            and os.environ.get("RTSEG_POOL", "1") != "0")


class _PoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, mode, cip):
        y, idx = ops().pool2d_fwd(x, k, s, p, mode, cip)
        ctx.geom = (x.shape[2], x.shape[3], k, s, p, mode, cip)
        if mode == _MAX:
            ctx.save_for_backward(idx)
            ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, gy):
        h, w, k, s, p, mode, cip = ctx.geom
        idx = ctx.saved_tensors[0] if mode == _MAX else gy.new_empty(0, dtype=torch.uint8)
        return ops().pool2d_bwd(gy, idx, h, w, k, s, p, mode, cip), None, None, None, None, None


class _AdaptiveAvgFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, oh, ow):
        ctx.geom = (x.shape[2], x.shape[3], x.is_contiguous(memory_format=torch.channels_last)
                    and not x.is_contiguous())
        return ops().adaptive_avg_pool_fwd(x, oh, ow)

    @staticmethod
    def backward(ctx, gy):
        h, w, cl = ctx.geom
        return ops().adaptive_avg_pool_bwd(gy, h, w, cl), None, None


class _MaxPoolIdxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx, win = ops().max_pool_indices(x, k, s, p)
        ctx.geom = (x.shape[2], x.shape[3], k, s, p)
        ctx.save_for_backward(win)
        ctx.mark_non_differentiable(idx)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the index output
        return y, idx

    @staticmethod
    def backward(ctx, gy, _gidx):
        if gy is None:
            return None, None, None, None
        h, w, k, s, p = ctx.geom
        (win,) = ctx.saved_tensors
        return ops().pool2d_bwd(gy, win, h, w, k, s, p, _MAX, True), None, None, None


class _UnpoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, idx, kh, kw, oh, ow):
        ctx.save_for_backward(idx)
        return ops().max_unpool_fwd(x, idx, kh, kw, oh, ow)

    @staticmethod
    def backward(ctx, gy):
        (idx,) = ctx.saved_tensors
        return ops().max_unpool_bwd(gy, idx), None, None, None, None, None


def max_pool2d_with_indices(x, kernel_size, stride=None, padding=0):
    """``F.max_pool2d(..., return_indices=True)``: (y, int64 flat plane indices)."""
    k = _pair(kernel_size)
    s = _pair(stride) if stride is not None else k
    p = _pair(padding)
    if _hip_ok(x) and 2 * p[0] <= k[0] and 2 * p[1] <= k[1] and k[0] * k[1] <= 256:
        return _MaxPoolIdxFn.apply(x, k, s, p)
    return F.max_pool2d(x, k, s, p, return_indices=True)


def max_unpool2d(x, indices, kernel_size, stride=None, padding=0, output_size=None):
    """``F.max_unpool2d`` -- gather form when kernel == stride and padding == 0 (the indices
    then come from a pool whose windows tile the plane)."""
    k = _pair(kernel_size)
    s = _pair(stride) if stride is not None else k
    p = _pair(padding)
    if output_size is not None:
        oh, ow = tuple(output_size)[-2:]
    else:
        oh, ow = (x.shape[2] - 1) * s[0] - 2 * p[0] + k[0], (x.shape[3] - 1) * s[1] - 2 * p[1] + k[1]
    if (_hip_ok(x) and k == s and p == (0, 0) and indices.dtype == torch.int64 and indices.shape == x.shape
            and indices.is_cuda):
        return _UnpoolFn.apply(x, indices, k[0], k[1], int(oh), int(ow))
    return F.max_unpool2d(x, indices, k, s, p, (oh, ow))


class _GlobalMaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y, idx = ops().global_max_pool(x)
        ctx.save_for_backward(idx)
        ctx.shape = x.shape
        ctx.fmt = torch.channels_last if (x.is_contiguous(memory_format=torch.channels_last)
                                          and not x.is_contiguous()) else torch.contiguous_format
        return y

    @staticmethod
    def backward(ctx, gy):
        (idx,) = ctx.saved_tensors
        n, c, h, w = ctx.shape
        gx = torch.zeros(ctx.shape, dtype=gy.dtype, device=gy.device).contiguous(memory_format=ctx.fmt)
        i = idx.view(n, c)
        nn_ = torch.arange(n, device=gy.device).view(n, 1).expand(n, c)
        cc = torch.arange(c, device=gy.device).view(1, c).expand(n, c)
        gx[nn_, cc, i // w, i % w] = gy.view(n, c)  # the max's gradient goes to its first argmax
        return gx


def adaptive_max_pool2d(x, output_size):
    """``F.adaptive_max_pool2d``; the global case (output 1x1) on the HIP kernel."""
    oh, ow = _pair(output_size)
    if (oh, ow) == (1, 1) and _hip_ok(x):
        return _GlobalMaxFn.apply(x)
    return F.adaptive_max_pool2d(x, (oh, ow))


def avg_pool2d(x, kernel_size, stride=None, padding=0, count_include_pad=True):
    """``F.avg_pool2d`` (ceil_mode False, no divisor override) on the HIP kernels."""
    k = _pair(kernel_size)
    s = _pair(stride) if stride is not None else k
    p = _pair(padding)
    if _hip_ok(x) and 2 * p[0] <= k[0] and 2 * p[1] <= k[1]:
        return _PoolFn.apply(x, k, s, p, _AVG, bool(count_include_pad))
    return F.avg_pool2d(x, k, s, p, count_include_pad=count_include_pad)


def max_pool2d(x, kernel_size, stride=None, padding=0):
    """``F.max_pool2d`` (dilation 1, ceil_mode False) on the HIP kernels."""
    k = _pair(kernel_size)
    s = _pair(stride) if stride is not None else k
    p = _pair(padding)
    if _hip_ok(x) and 2 * p[0] <= k[0] and 2 * p[1] <= k[1] and k[0] * k[1] <= 256:
        return _PoolFn.apply(x, k, s, p, _MAX, True)
    return F.max_pool2d(x, k, s, p)


def adaptive_avg_pool2d(x, output_size):
    """``F.adaptive_avg_pool2d`` on the HIP kernels (global pool = 2-stage reduction)."""
    oh, ow = _pair(output_size)
    oh = x.shape[2] if oh is None else oh
    ow = x.shape[3] if ow is None else ow
    if _hip_ok(x):
        return _AdaptiveAvgFn.apply(x, oh, ow)
    return F.adaptive_avg_pool2d(x, (oh, ow))


class AvgPool2d(nn.AvgPool2d):
    def forward(self, x):
        return avg_pool2d(x, self.kernel_size, self.stride, self.padding, self.count_include_pad)


class MaxPool2d(nn.MaxPool2d):
    def forward(self, x):
        if self.return_indices:
            return max_pool2d_with_indices(x, self.kernel_size, self.stride, self.padding)
        return max_pool2d(x, self.kernel_size, self.stride, self.padding)


class MaxUnpool2d(nn.MaxUnpool2d):
    def forward(self, x, indices, output_size=None):
        return max_unpool2d(x, indices, self.kernel_size, self.stride, self.padding, output_size)


class AdaptiveAvgPool2d(nn.AdaptiveAvgPool2d):
    def forward(self, x):
        return adaptive_avg_pool2d(x, self.output_size)


class AdaptiveMaxPool2d(nn.AdaptiveMaxPool2d):
    def forward(self, x):
        if self.return_indices:
            return nn.AdaptiveMaxPool2d.forward(self, x)
        return adaptive_max_pool2d(x, self.output_size)


def convert_pooling(model: nn.Module) -> nn.Module:
    """Swap eligible ``nn.AvgPool2d`` / ``nn.MaxPool2d`` / ``nn.AdaptiveAvgPool2d`` modules
    to their HIP-backed subclasses (in place)."""
    for m in model.modules():
        t = type(m)
        if t is nn.AvgPool2d and not m.ceil_mode and m.divisor_override is None:
            m.__class__ = AvgPool2d
        elif t is nn.MaxPool2d and not m.ceil_mode and _pair(m.dilation) == (1, 1):
            m.__class__ = MaxPool2d
        elif t is nn.MaxUnpool2d:
            m.__class__ = MaxUnpool2d
        elif t is nn.AdaptiveAvgPool2d:
            m.__class__ = AdaptiveAvgPool2d
        elif t is nn.AdaptiveMaxPool2d:
            m.__class__ = AdaptiveMaxPool2d
    return model
