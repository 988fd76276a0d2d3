"""STDC detail loss (Laplacian detail target + Dice + BCE) on the fused HIP kernels of
``csrc/kernels/detail_loss.hip``.

Reference: core/seg_trainer.py:68-82 (target construction and the x8 bilinear resize of the
detail logits), core/loss.py:23-52 (Dice on RAW logits + BCE-with-logits) and
models/stdc.py:131-147 (3-scale Laplacian of the label map).  :func:`detail_loss` takes the
low-resolution detail logits and the label map and returns the scalar loss; on GPU the whole
chain is one forward kernel (+ finalize) and one backward kernel + the separable bilinear
backward, on CPU it is the PyTorch formulation of the reference.  The target is computed in
fp32 from the integer labels (exact; the reference computes it under autocast).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import ops, use_hip


class _DetailLossFn(torch.autograd.Function):
    """Fused detail loss.  ``weight`` / ``bias`` are the LIVE ``detail_conv`` parameters: the
    thresholded target is piecewise constant in them, so their gradient is exactly zero -- but
    it is a real zero gradient, as in the reference (core/seg_trainer.py:74-76, where
    detail_conv runs inside the graph): SGD weight decay and momentum then act on detail_conv
    every step, and DDP sees the parameter as used."""

    @staticmethod
    def forward(ctx, d, labels, weight, bias, thrs, dice_coef, bce_coef):
        w = weight.detach().reshape(-1).float()
        b = bias.detach().reshape(-1).float() if bias is not None else w.new_zeros(1)
        wb = torch.cat([w, b]).contiguous()
        loss, y, sums = ops().detail_loss_fwd(d, labels, wb, thrs, dice_coef, bce_coef)
        ctx.save_for_backward(d, y, sums)
        ctx.coefs = (dice_coef, bce_coef)
        ctx.wshape = (weight.shape, weight.dtype, None if bias is None else (bias.shape, bias.dtype))
        ctx.mark_non_differentiable(y, sums)
        return loss

    @staticmethod
    def backward(ctx, g):
        d, y, sums = ctx.saved_tensors
        gd = ops().detail_loss_bwd(g, d, y, sums, *ctx.coefs)
        (ws, wdt, bsd) = ctx.wshape
        gw = torch.zeros(ws, dtype=wdt, device=d.device) if ctx.needs_input_grad[2] else None
        gb = torch.zeros(bsd[0], dtype=bsd[1], device=d.device) if bsd is not None and ctx.needs_input_grad[3] else None
        return gd, None, gw, gb, None, None, None


def detail_target_reference(labels: torch.Tensor, detail_conv: nn.Module, thrs: float, laplacian=None):
    """Binary detail target [N, 1, H, W] (fp32), the reference's construction."""
    if laplacian is None:
        from ..models.stdc import LaplacianConv

        laplacian = LaplacianConv()
    gt = laplacian(labels.unsqueeze(1).float())
    gt = F.conv2d(gt, detail_conv.weight.float(), None if detail_conv.bias is None else detail_conv.bias.float())
    # the reference thresholds in place on the graph (core/seg_trainer.py:74-76): detail_conv
    # stays connected with an exactly-zero gradient -- `gt * 0 + mask` keeps that
    return gt * 0.0 + (gt.detach() > thrs).float()


def detail_loss_reference(detail_logits, labels, detail_conv, thrs, dice_coef=1.0, bce_coef=1.0, laplacian=None):
    from ..core.loss import DetailLoss

    gt = detail_target_reference(labels, detail_conv, thrs, laplacian)
    p = F.interpolate(detail_logits, gt.shape[2:], mode="bilinear", align_corners=True)
    return DetailLoss(dice_coef, bce_coef)(p.float(), gt)


def detail_loss(detail_logits: torch.Tensor, labels: torch.Tensor, detail_conv: nn.Module, thrs: float,
                dice_coef: float = 1.0, bce_coef: float = 1.0, laplacian=None) -> torch.Tensor:
    """Detail loss from the H/8 detail logits ``[N, 1, h, w]`` and labels ``[N, H, W]``."""
    if use_hip(detail_logits, "detail") and labels.dtype in (torch.uint8, torch.int64):
        return _DetailLossFn.apply(detail_logits, labels.contiguous(), detail_conv.weight, detail_conv.bias,
                                   float(thrs), float(dice_coef), float(bce_coef))
    return detail_loss_reference(detail_logits, labels, detail_conv, thrs, dice_coef, bce_coef, laplacian)
