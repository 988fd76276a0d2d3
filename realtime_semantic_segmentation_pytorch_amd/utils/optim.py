"""Optimizer, LR scheduler and model EMA.

Parity: reference utils/optimizer.py:4-20 (SGD lr = base_lr * gpu_num with
momentum/weight decay; Adam/AdamW lr = 1e-3 * gpu_num, no weight decay),
utils/scheduler.py:5-25 (per-iteration OneCycleLR 'cos_warmup' / 'linear',
StepLR 'step'), utils/model_ema.py:12-40 (EMA over the full state dict with the
decay ramp ``cur_itrs / total_itrs``, or a plain copy when ``use_ema=False``).

MI355X: optimizers use the multi-tensor (``foreach``) paths so one step is a
handful of launches; the EMA update is a single multi-tensor lerp/copy over
pre-gathered tensor lists (no per-step ``state_dict()`` walk).
"""
from __future__ import annotations

from copy import deepcopy
from math import ceil

import torch
import torch.nn as nn
from torch.optim import SGD, Adam, AdamW
from torch.optim.lr_scheduler import OneCycleLR, StepLR

from ..parallel import de_parallel


def get_optimizer(config, model):
    params = [p for p in model.parameters() if p.requires_grad]
    on_gpu = bool(params) and params[0].is_cuda
    if config.optimizer_type == "sgd":
        config.lr = config.base_lr * config.gpu_num
        return SGD(params, lr=config.lr, momentum=config.momentum,
                   weight_decay=config.weight_decay, foreach=on_gpu)
    if config.optimizer_type in ("adam", "adamw"):
        config.lr = 0.001 * config.gpu_num
        cls = Adam if config.optimizer_type == "adam" else AdamW
        kw = {"foreach": on_gpu}
        if cls is AdamW:
            kw["weight_decay"] = 0.01  # torch default, as the reference passes none
        return cls(params, lr=config.lr, **kw)
    raise NotImplementedError(f"Unsupported optimizer type: {config.optimizer_type}")


def get_scheduler(config, optimizer, iters_per_epoch=None):
    if iters_per_epoch is None:
        denom = config.train_bs * (config.gpu_num if config.DDP else 1)
        iters_per_epoch = ceil(config.train_num / denom)
    config.iters_per_epoch = max(1, int(iters_per_epoch))
    config.total_itrs = int(config.total_epoch * config.iters_per_epoch)
    if config.lr_policy == "cos_warmup":
        return OneCycleLR(optimizer, max_lr=config.lr, total_steps=config.total_itrs,
                          pct_start=min(float(config.warmup_epochs) / config.total_epoch, 0.99))
    if config.lr_policy == "linear":
        return OneCycleLR(optimizer, max_lr=config.lr, total_steps=config.total_itrs,
                          pct_start=0.0, anneal_strategy="linear")
    if config.lr_policy == "step":
        return StepLR(optimizer, step_size=config.step_size * config.iters_per_epoch, gamma=0.1)
    raise NotImplementedError(f"Unsupported scheduler type: {config.lr_policy}")


class ModelEmaV2(nn.Module):
    def __init__(self, config, model, device=None):
        super().__init__()
        self.ema = deepcopy(de_parallel(model)).eval()
        for p in self.ema.parameters():
            p.requires_grad_(False)
        self.device = device
        if device is not None:
            self.ema.to(device=device)
        self.use_ema = config.use_ema
        self.total_itrs = max(1, int(getattr(config, "total_itrs", 1)))
        self._pairs = None
        self._src_id = None

    def _gather(self, model):
        src = de_parallel(model)
        if self._pairs is None or self._src_id != id(src):
            e_sd, m_sd = self.ema.state_dict(), src.state_dict()
            fe, fm, ie, im = [], [], [], []
            for k, ev in e_sd.items():
                mv = m_sd[k]
                if ev.is_floating_point():
                    fe.append(ev); fm.append(mv)
                else:
                    ie.append(ev); im.append(mv)
            self._pairs = (fe, fm, ie, im)
            self._src_id = id(src)
        return self._pairs

    @torch.no_grad()
    def update(self, model, cur_itrs):
        fe, fm, ie, im = self._gather(model)
        if self.use_ema:
            decay = min(max(cur_itrs / self.total_itrs, 0.0), 1.0)
            # e = decay*e + (1-decay)*m  ==  lerp(e, m, 1-decay)
            torch._foreach_lerp_(fe, fm, 1.0 - decay)
        else:
            torch._foreach_copy_(fe, fm)
        if ie:
            torch._foreach_copy_(ie, im)

    def set_model(self, model):
        self.ema = deepcopy(de_parallel(model)).eval()
        self._pairs = None


def get_ema_model(config, model, device):
    return ModelEmaV2(config, model, device=device)
