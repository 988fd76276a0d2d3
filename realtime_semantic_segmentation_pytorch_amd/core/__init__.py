from .base_trainer import BaseTrainer
from .seg_trainer import SegTrainer
from .loss import (get_loss_fn, get_detail_loss_fn, kd_loss_fn, OhemCELoss, SegCELoss, DiceLoss,
                   DetailLoss)

__all__ = ["BaseTrainer", "SegTrainer", "get_loss_fn", "get_detail_loss_fn", "kd_loss_fn",
           "OhemCELoss", "SegCELoss", "DiceLoss", "DetailLoss"]
