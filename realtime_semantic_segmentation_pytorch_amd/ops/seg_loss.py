"""Fused segmentation cross-entropy / OHEM (HIP kernel ``seg_loss.hip``).

``seg_cross_entropy(logits, labels, ...)`` evaluates the loss on the label
grid.  ``logits`` may be at a lower resolution than ``labels`` (the model's
final bilinear upsample is then applied inside the kernel) or at a different
resolution than the labels with ``label_mode='nearest'`` semantics (the
aux-head path of reference core/seg_trainer.py:57-62).

CPU tensors use the literal PyTorch formulation of reference core/loss.py:6-20
(OHEM) and core/loss.py:61-63 (CE), which is also the test oracle.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from ._ext import use_hip, ops

MODE_OHEM, MODE_MEAN, MODE_SUM = 0, 1, 2


class _SegLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, out_h, out_w, align, ignore, cw, mode, thresh):
        loss, pix_loss, pix_lse, stats = ops().seg_loss_fwd(
            logits, labels, out_h, out_w, align, ignore, cw, mode, thresh)
        ctx.save_for_backward(logits, labels, pix_loss, pix_lse, stats, cw)
        ctx.cfg = (out_h, out_w, align, ignore, mode)
        return loss

    @staticmethod
    def backward(ctx, g):
        logits, labels, pix_loss, pix_lse, stats, cw = ctx.saved_tensors
        out_h, out_w, align, ignore, mode = ctx.cfg
        gl = ops().seg_loss_bwd(g, logits, labels, pix_loss, pix_lse, stats, out_h, out_w, align,
                                ignore, cw, mode)
        return gl, None, None, None, None, None, None, None, None


def _resize_labels_nearest(labels: torch.Tensor, size) -> torch.Tensor:
    if tuple(labels.shape[-2:]) == tuple(size):
        return labels
    lab = F.interpolate(labels.unsqueeze(1).float(), size, mode="nearest")
    return lab.squeeze(1).long()


def _fused_ok(logits: torch.Tensor, out_hw) -> bool:
    c = logits.shape[1]
    h, w = logits.shape[2], logits.shape[3]
    if c > 256:
        return False
    if (h, w) == tuple(out_hw):
        return True
    # upsample only: the backward keeps a [C, TH, TW] gradient tile in LDS (seg_loss.hip)
    return h <= out_hw[0] and w <= out_hw[1]


def seg_cross_entropy(logits: torch.Tensor, labels: torch.Tensor, *, mode: int = MODE_OHEM,
                      ohem_thrs: float = 0.7, ignore_index: int = 255,
                      class_weight: Optional[torch.Tensor] = None,
                      out_size: Optional[Tuple[int, int]] = None, align_corners: bool = True,
                      resize_logits: bool = True) -> torch.Tensor:
    """Cross-entropy (OHEM / mean / sum) of ``logits`` against ``labels``.

    * ``resize_logits=True``: logits are bilinearly resized to ``out_size``
      (default: the label size) -- the model-output path.
    * ``resize_logits=False``: the loss is taken at logit resolution and labels
      are nearest-resized to it -- the aux-head path.
    """
    if labels.dim() == 4:
        labels = labels.squeeze(1)
    if labels.dtype not in (torch.int64, torch.uint8):
        labels = labels.long()
    if out_size is None:
        out_size = tuple(labels.shape[-2:]) if resize_logits else tuple(logits.shape[-2:])
    out_size = (int(out_size[0]), int(out_size[1]))
    thresh = -math.log(ohem_thrs)
    if use_hip(logits, "loss") and logits.dtype in (torch.float32, torch.bfloat16, torch.float16):
        if not resize_logits:
            out_size = tuple(logits.shape[-2:])
        if _fused_ok(logits, out_size):
            cw = class_weight.float().contiguous() if class_weight is not None else None
            return _SegLossFn.apply(logits, labels.contiguous(), out_size[0], out_size[1],
                                    bool(align_corners), int(ignore_index), cw, int(mode), thresh)
        logits = F.interpolate(logits, out_size, mode="bilinear", align_corners=align_corners)
        cw = class_weight.float().contiguous() if class_weight is not None else None
        return _SegLossFn.apply(logits, labels.contiguous(), out_size[0], out_size[1],
                                bool(align_corners), int(ignore_index), cw, int(mode), thresh)
    return seg_cross_entropy_reference(logits, labels.long(), mode=mode, ohem_thrs=ohem_thrs,
                                       ignore_index=ignore_index, class_weight=class_weight,
                                       out_size=out_size, align_corners=align_corners,
                                       resize_logits=resize_logits)


def seg_cross_entropy_reference(logits, labels, *, mode=MODE_OHEM, ohem_thrs=0.7, ignore_index=255,
                                class_weight=None, out_size=None, align_corners=True,
                                resize_logits=True):
    """Plain-PyTorch formulation (CPU path and numerics oracle)."""
    if labels.dim() == 4:
        labels = labels.squeeze(1)
    labels = labels.long()
    if resize_logits:
        if out_size is None:
            out_size = tuple(labels.shape[-2:])
        if tuple(logits.shape[-2:]) != tuple(out_size):
            logits = F.interpolate(logits, out_size, mode="bilinear", align_corners=align_corners)
        labels = _resize_labels_nearest(labels, out_size)
    else:
        labels = _resize_labels_nearest(labels, logits.shape[-2:])
    logits = logits.float()
    if mode == MODE_OHEM:
        thresh = -math.log(ohem_thrs)
        n_min = int((labels != ignore_index).sum().item()) // 16
        loss = F.cross_entropy(logits, labels, ignore_index=ignore_index, reduction="none").view(-1)
        hard = loss[loss > thresh]
        if hard.numel() < n_min:
            hard, _ = loss.topk(n_min)
        if hard.numel() == 0:
            return loss.sum() * 0.0
        return hard.mean()
    red = "mean" if mode == MODE_MEAN else "sum"
    w = class_weight.float().to(logits.device) if class_weight is not None else None
    return F.cross_entropy(logits, labels, weight=w, ignore_index=ignore_index, reduction=red)
