"""Knowledge-distillation KL loss (reference core/loss.py:80-88).

``T^2 * mean_{n,c,h,w}( p_t * (log p_t - log p_s) )`` with ``p = softmax(z / T)``
over the class dim -- i.e. ``F.kl_div(log_softmax(s/T), softmax(t/T)) * T**2``
with the default element-mean reduction.  GPU tensors use the fused HIP kernel
(one max pass + one exp pass per pixel; per-pixel log-sum-exps are kept for
the single-pass backward ``(p_s - p_t) * T / numel``; kernels in
``csrc/kernels/kd_metrics.hip``).
"""
from __future__ import annotations

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


def kd_kl_div_reference(s: torch.Tensor, t: torch.Tensor, temperature: float) -> torch.Tensor:
    T = float(temperature)
    # == F.kl_div(log_softmax(s/T), softmax(t/T)) * T^2 with the default element-mean reduction
    lt = F.log_softmax(t.float() / T, dim=1)
    return (lt.exp() * (lt - F.log_softmax(s.float() / T, dim=1))).mean() * T ** 2


def kd_kl_div(s: torch.Tensor, t: torch.Tensor, temperature: float) -> torch.Tensor:
    if use_hip(s, "kd") and s.dim() == 4 and s.shape == t.shape and s.dtype in (torch.float32, torch.bfloat16,
                                                                           torch.float16):
        return _KDFn.apply(s, t.detach().to(s.dtype), float(temperature))
    return kd_kl_div_reference(s, t, temperature)
