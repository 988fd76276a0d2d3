"""Objectives (parity: reference core/loss.py:6-88).

* :class:`OhemCELoss` / ``loss_type='ohem'`` and ``loss_type='ce'`` run on the
  fused HIP kernel (``ops.seg_cross_entropy``): per-pixel CE + OHEM selection on
  device without host syncs, optionally consuming head-resolution logits
  (``DeferredLogits``) so the final upsample is folded into the loss.
* :func:`kd_loss_fn` -- Hinton KD (KL with the reference's element-mean
  reduction x T^2, or MSE) on the fused HIP KL kernel when available.
* :class:`DiceLoss`, :class:`DetailLoss` -- STDC detail supervision.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..ops.interp import DeferredLogits


class SegCELoss(nn.Module):
    """CE/OHEM on full-resolution labels; accepts tensors or :class:`DeferredLogits`."""

    def __init__(self, mode=ops.MODE_OHEM, thresh=0.7, ignore_index=255, weight=None):
        super().__init__()
        self.mode = mode
        self.thresh = thresh
        self.ignore_index = ignore_index
        if weight is not None:
            self.register_buffer("weight", torch.as_tensor(weight, dtype=torch.float32))
        else:
            self.weight = None

    def forward(self, logits, labels):
        if isinstance(logits, DeferredLogits):
            return ops.seg_cross_entropy(logits.logits, labels, mode=self.mode,
                                         ohem_thrs=self.thresh, ignore_index=self.ignore_index,
                                         class_weight=self.weight, out_size=logits.size,
                                         align_corners=logits.align_corners, resize_logits=True)
        return ops.seg_cross_entropy(logits, labels, mode=self.mode, ohem_thrs=self.thresh,
                                     ignore_index=self.ignore_index, class_weight=self.weight,
                                     resize_logits=True)

    def aux(self, logits, labels):
        """Aux-head loss: evaluated at head resolution against nearest-resized labels."""
        return ops.seg_cross_entropy(logits, labels, mode=self.mode, ohem_thrs=self.thresh,
                                     ignore_index=self.ignore_index, class_weight=self.weight,
                                     resize_logits=False)


class OhemCELoss(SegCELoss):
    """Reference-named OHEM loss (threshold given as a probability, like the reference)."""

    def __init__(self, thresh, ignore_index=255):
        super().__init__(ops.MODE_OHEM, thresh, ignore_index)
        self.thresh_logit = -math.log(thresh)


class DiceLoss(nn.Module):
    """1 - (2 sum(p*y) + s) / (sum p + sum y + s) per sample on RAW logits (reference :23-35)."""

    def __init__(self, smooth=1):
        super().__init__()
        self.smooth = smooth

    def forward(self, logits, labels):
        p = logits.flatten(1)
        y = labels.flatten(1)
        inter = (p * y).sum(1)
        return (1 - (2 * inter + self.smooth) / (p.sum(1) + y.sum(1) + self.smooth)).mean()


class DetailLoss(nn.Module):
    """STDC detail loss = dice_coef * Dice + bce_coef * BCE-with-logits (reference :38-52)."""

    def __init__(self, dice_loss_coef=1.0, bce_loss_coef=1.0, smooth=1):
        super().__init__()
        self.dice_loss_coef = dice_loss_coef
        self.bce_loss_coef = bce_loss_coef
        self.dice_loss_fn = DiceLoss(smooth)
        self.bce_loss_fn = nn.BCEWithLogitsLoss()

    def forward(self, logits, labels):
        return (self.dice_loss_coef * self.dice_loss_fn(logits, labels)
                + self.bce_loss_coef * self.bce_loss_fn(logits, labels))


def get_loss_fn(config, device=None):
    weights = None if config.class_weights is None else list(
        config.class_weights if isinstance(config.class_weights, (list, tuple)) else [config.class_weights])
    if config.loss_type == "ce":
        red = getattr(config, "reduction", "mean")
        if red not in ("mean", "sum"):
            raise NotImplementedError(f"Unsupported CE reduction: {red}")
        fn = SegCELoss(ops.MODE_MEAN if red == "mean" else ops.MODE_SUM, config.ohem_thrs,
                       config.ignore_index, weights)
    elif config.loss_type == "ohem":
        fn = SegCELoss(ops.MODE_OHEM, config.ohem_thrs, config.ignore_index, None)
    else:
        raise NotImplementedError(f"Unsupport loss type: {config.loss_type}")
    return fn.to(device) if device is not None else fn


def get_detail_loss_fn(config):
    return DetailLoss(dice_loss_coef=config.dice_loss_coef, bce_loss_coef=config.bce_loss_coef)


def kd_loss_fn(config, outputs, outputsT):
    """Knowledge-distillation loss between student and (detached) teacher logits."""
    outputsT = ops.materialize(outputsT).detach()
    if config.kd_loss_type == "kl_div":  # (deferred student logits: the upsample folds into the KD kernels)
        return ops.kd_kl_div(outputs, outputsT, config.kd_temperature)
    outputs = ops.materialize(outputs)
    if config.kd_loss_type == "mse":
        return F.mse_loss(outputs, outputsT)
    raise NotImplementedError(f"Unsupported kd loss type: {config.kd_loss_type}")
