"""Optimizer, LR scheduler and model EMA.

Parity: reference utils/optimizer.py:4-20 (SGD lr = base_lr * gpu_num with
momentum/weight decay; Adam/AdamW lr = 1e-3 * gpu_num, no weight decay),
utils/scheduler.py:5-25 (per-iteration OneCycleLR 'cos_warmup' / 'linear',
StepLR 'step'), utils/model_ema.py:12-40 (EMA over the full state dict with the
decay ramp ``cur_itrs / total_itrs``, or a plain copy when ``use_ema=False``).

MI355X: on GPU the optimizers are ``ops.FusedSGD / FusedAdam / FusedAdamW``
(torch-compatible state, one HIP launch per step) and the EMA of every
parameter is written by that same launch (``ModelEmaV2.attach``); only the BN
running statistics are lerped separately (one more launch).  CPU runs use the
torch ``foreach`` paths and a multi-tensor lerp over pre-gathered tensor lists
(no per-step ``state_dict()`` walk).
"""
from __future__ import annotations

from copy import deepcopy
from math import ceil

import torch
import torch.nn as nn
from torch.optim import SGD, Adam, AdamW
from torch.optim.lr_scheduler import OneCycleLR, StepLR

from ..parallel import de_parallel
from ..ops.optim import FusedAdam, FusedAdamW, FusedSGD, ema_lerp_


def get_optimizer(config, model):
    params = [p for p in model.parameters() if p.requires_grad]
    on_gpu = bool(params) and params[0].is_cuda
    fused = on_gpu and bool(getattr(config, "fused_optimizer", True))
    if config.optimizer_type == "sgd":
        config.lr = config.base_lr * config.gpu_num
        return (FusedSGD if fused else SGD)(params, lr=config.lr, momentum=config.momentum,
                                            weight_decay=config.weight_decay, foreach=on_gpu)
    if config.optimizer_type in ("adam", "adamw"):
        config.lr = 0.001 * config.gpu_num
        if config.optimizer_type == "adam":
            cls = FusedAdam if fused else Adam
        else:
            cls = FusedAdamW if fused else AdamW
        kw = {"foreach": on_gpu}
        if config.optimizer_type == "adamw":
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
        self._fused_opt = None

    def _gather(self, model):
        src = de_parallel(model)
        if self._pairs is None or self._src_id != id(src):
            e_sd, m_sd = self.ema.state_dict(), src.state_dict()
            pnames = {n for n, _ in src.named_parameters()}
            pe, pm, be, bm, ie, im = [], [], [], [], [], []
            for k, ev in e_sd.items():
                mv = m_sd[k]
                if not ev.is_floating_point():
                    ie.append(ev); im.append(mv)
                elif k in pnames:
                    pe.append(ev); pm.append(mv)
                else:
                    be.append(ev); bm.append(mv)
            self._pairs = (pe, pm, be, bm, ie, im)
            self._src_id = id(src)
        return self._pairs

    def decay(self, cur_itrs):
        return min(max(cur_itrs / self.total_itrs, 0.0), 1.0) if self.use_ema else 0.0

    def attach(self, optimizer, model):
        """Let a fused optimizer write the EMA of every parameter inside its step."""
        if not hasattr(optimizer, "attach_ema"):
            return False
        src = de_parallel(model)
        e_named = dict(self.ema.named_parameters())
        pairs = [(p, e_named[n].data) for n, p in src.named_parameters() if n in e_named]
        optimizer.attach_ema(pairs)
        self._fused_opt = optimizer
        return True

    @torch.no_grad()
    def update(self, model, cur_itrs, params_done=False):
        """EMA after one optimizer step. ``params_done``: the fused optimizer already wrote the
        parameter EMAs with this step's decay, only buffers remain."""
        pe, pm, be, bm, ie, im = self._gather(model)
        w = 1.0 - self.decay(cur_itrs)  # e = decay*e + (1-decay)*m == lerp(e, m, 1-decay)
        groups = [(be, bm)] if params_done else [(pe, pm), (be, bm)]
        for fe, fm in groups:
            if not fe:
                continue
            if fe[0].is_cuda and fe[0].dtype == torch.float32 and all(
                    t.dtype == torch.float32 and t.is_contiguous() for t in fe + fm):
                ema_lerp_(list(zip(fm, fe)), w)
            elif w >= 1.0:
                torch._foreach_copy_(fe, fm)
            else:
                torch._foreach_lerp_(fe, fm, w)
        if ie:
            torch._foreach_copy_(ie, im)

    def set_model(self, model):
        self.ema = deepcopy(de_parallel(model)).eval()
        self._pairs = None
        if getattr(self, "_fused_opt", None) is not None:
            self._fused_opt.attach_ema([])
            self._fused_opt = None


def get_ema_model(config, model, device):
    return ModelEmaV2(config, model, device=device)
