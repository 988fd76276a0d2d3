"""Confusion matrix of argmax predictions (reference utils/metrics.py via torchmetrics).

``confusion_matrix(logits[N,C,H,W] | labels[N,H,W], target[N,H,W], C, ignore)``
returns ``cm[target, pred]`` as int64 ``[C, C]``.  GPU: one HIP kernel fusing the
class argmax with an LDS-private histogram (``csrc/kernels/kd_metrics.hip``); CPU: bincount.
"""
from __future__ import annotations

import torch

from ._ext import use_hip, ops


def confusion_matrix_reference(preds, target, num_class, ignore_index=255):
    if preds.dim() == 4:
        preds = preds.argmax(1)
    target = target.long()
    keep = (target != ignore_index) & (target >= 0) & (target < num_class)
    idx = target[keep] * num_class + preds[keep].long()
    return torch.bincount(idx, minlength=num_class * num_class).reshape(num_class, num_class)


def confusion_matrix(preds, target, num_class, ignore_index=255):
    if (use_hip(preds) and preds.dim() == 4
            and preds.dtype in (torch.float32, torch.bfloat16, torch.float16)):
        return ops().confmat(preds, target.long().contiguous(), num_class, ignore_index)
    return confusion_matrix_reference(preds, target, num_class, ignore_index)
