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
Unsupported variants (``ceil_mode``, ``divisor_override``, dilation,
``return_indices``) keep the PyTorch module.  ``RTSEG_POOL=0`` disables the path
for A/B comparisons.
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
    return (x.dim() == 4 and x.dtype in _DTYPES and x.numel() < 2 ** 31 and use_hip(x)
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
        return max_pool2d(x, self.kernel_size, self.stride, self.padding)


class AdaptiveAvgPool2d(nn.AdaptiveAvgPool2d):
    def forward(self, x):
        return adaptive_avg_pool2d(x, self.output_size)


def convert_pooling(model: nn.Module) -> nn.Module:
    """Swap eligible ``nn.AvgPool2d`` / ``nn.MaxPool2d`` / ``nn.AdaptiveAvgPool2d`` modules
    to their HIP-backed subclasses (in place)."""
    for m in model.modules():
        t = type(m)
        if t is nn.AvgPool2d and not m.ceil_mode and m.divisor_override is None:
            m.__class__ = AvgPool2d
        elif (t is nn.MaxPool2d and not m.ceil_mode and not m.return_indices
              and _pair(m.dilation) == (1, 1)):
            m.__class__ = MaxPool2d
        elif t is nn.AdaptiveAvgPool2d:
            m.__class__ = AdaptiveAvgPool2d
    return model
