"""Knowledge-distillation KL loss (reference core/loss.py:80-88).

``T^2 * mean_{n,c,h,w}( p_t * (log p_t - log p_s) )`` with ``p = softmax(z / T)``
over the class dim -- i.e. ``F.kl_div(log_softmax(s/T), softmax(t/T)) * T**2``
with the default element-mean reduction.  GPU tensors use the fused HIP kernel
(one max pass + one exp pass per pixel; per-pixel log-sum-exps are kept for
the single-pass backward ``(p_s - p_t) * T / numel``; kernels in
``csrc/kernels/kd_metrics.hip``).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ._ext import use_hip, ops


class _KDFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, t, temperature):
        loss, lse = ops().kd_kl_fwd(s, t, temperature)
        ctx.save_for_backward(s, t, lse)
        ctx.temperature = temperature
        return loss

    @staticmethod
    def backward(ctx, g):
        s, t, lse = ctx.saved_tensors
        return ops().kd_kl_bwd(g, s, t, lse, ctx.temperature), None, None


class _KDFoldFn(torch.autograd.Function):
    """KD on the student's HEAD-resolution logits ``lo`` with the model's final bilinear upsample to
    the teacher's size folded into the loss kernels: the full-resolution student logits are never
    materialised (forward), and the backward writes their gradient once for the upsample's backward
    (``interp_backward``) to map down -- the trainer's fused CE loss does the same with its labels."""

    @staticmethod
    def forward(ctx, lo, t, temperature, align):
        loss, lse = ops().kd_kl_fwd_fold(lo, t, temperature, align)
        ctx.save_for_backward(lo, t, lse)
        ctx.temperature, ctx.align = temperature, align
        return loss

    @staticmethod
    def backward(ctx, g):
        lo, t, lse = ctx.saved_tensors
        gs = ops().kd_kl_bwd_fold(g, lo, t, lse, ctx.temperature, ctx.align)
        glo = ops().interp_backward(gs, lo.shape[2], lo.shape[3], ctx.align, True)
        return glo.to(lo.dtype), None, None, None


def _fold_ok(lo: torch.Tensor, t: torch.Tensor) -> bool:
    return (lo.dim() == 4 and t.dim() == 4 and lo.shape[:2] == t.shape[:2] and lo.dtype == t.dtype
            and lo.dtype in (torch.float32, torch.bfloat16, torch.float16)
            and lo.is_contiguous(memory_format=torch.channels_last) and t.is_contiguous(memory_format=torch.channels_last)
            and lo.data_ptr() % 16 == 0 and t.data_ptr() % 16 == 0)


def kd_kl_div_reference(s: torch.Tensor, t: torch.Tensor, temperature: float) -> torch.Tensor:
    T = float(temperature)
    # == F.kl_div(log_softmax(s/T), softmax(t/T)) * T^2 with the default element-mean reduction
    lt = F.log_softmax(t.float() / T, dim=1)
    return (lt.exp() * (lt - F.log_softmax(s.float() / T, dim=1))).mean() * T ** 2


def kd_kl_div(s, t: torch.Tensor, temperature: float) -> torch.Tensor:
    """``s``: student logits, or the trainer's :class:`DeferredLogits` (head resolution + the final
    upsample) -- folded into the kernels on the GPU when the layouts allow, else materialised."""
    from .interp import DeferredLogits

    if isinstance(s, DeferredLogits):
        lo = s.logits
        if (use_hip(lo, "kd") and tuple(t.shape[2:]) == s.size and tuple(lo.shape[2:]) != s.size
                and os.environ.get("RTSEG_KD_FOLD", "1") != "0"):
            tt = t.detach().to(lo.dtype)
            if _fold_ok(lo, tt):
                return _KDFoldFn.apply(lo, tt, float(temperature), bool(s.align_corners))
        s = s.materialize()
    if use_hip(s, "kd") and s.dim() == 4 and s.shape == t.shape and s.dtype in (torch.float32, torch.bfloat16,
                                                                           torch.float16):
        return _KDFn.apply(s, t.detach().to(s.dtype), float(temperature))
    return kd_kl_div_reference(s, t, temperature)
