"""Trainer lifecycle (parity: reference core/base_trainer.py:14-186).

Same flow -- env-derived DDP flag, logger, device + process group, AMP, seed,
model, loaders, optimizer, scheduler, auto-resume from ``{save_dir}/last.pth``,
EMA, epoch loop with validation/best/last checkpoints, ``val_best`` -- and the
same checkpoint format (``cur_epoch, best_score, state_dict, optimizer,
scheduler``; best.pth holds EMA weights with optimizer/scheduler ``None``).

Fixes: ``save_ckpt`` with ``ckpt_name`` (#11), a barrier after
rank-0 checkpoint writes before other ranks read them (#12), scheduler length
from the real loader (#23); extra keys ``ema_state_dict`` / ``scaler`` are
stored in last.pth so a resume restores EMA and the fp16 loss scale too.
"""
from __future__ import annotations

import os

import torch

from ..datasets import get_loader, get_test_loader
from ..models import get_model
from ..parallel import barrier, dist_env
from ..utils import (de_parallel, destroy_ddp_process, get_ema_model, get_logger, get_optimizer,
                     get_scheduler, get_writer, log_config, mkdir, parallel_model, save_config,
                     set_device, set_seed)
from ..utils.runtime import configure_backend
from .loss import get_loss_fn


def inject_fault(epoch: int):
    """Failure injection for restart tests (tests/test_elastic_cpu.py): with
    ``RTSEG_FAULT_EPOCH=e`` and ``RTSEG_FAULT_SENTINEL=path``, the LAST rank dies (exit 17) when
    epoch ``e`` starts -- once: the sentinel file marks that the fault has fired, so the restarted
    job (torchrun ``--max-restarts``) resumes from ``last.pth`` and runs through."""
    want, sentinel = os.environ.get("RTSEG_FAULT_EPOCH"), os.environ.get("RTSEG_FAULT_SENTINEL")
    if want is None or sentinel is None or int(want) != epoch or os.path.exists(sentinel):
        return
    rank, _, world = dist_env()
    if rank == max(world - 1, 0) or rank == -1:
        with open(sentinel, "w") as f:
            f.write(f"rank {rank} killed at epoch {epoch}\n")
        os._exit(17)


class BaseTrainer:
    def __init__(self, config):
        self.rank, self.local_rank, self.world_size = dist_env()
        config.DDP = self.local_rank != -1
        self.main_rank = self.local_rank in (-1, 0) and self.rank in (-1, 0)
        if hasattr(config, "init_dependent_config"):
            config.init_dependent_config()  # idempotent; main.py calls it too
        self.logger = get_logger(config, self.main_rank)
        # same find-mode policy as bench.py (which alone also drops the naive solvers)
        configure_backend(getattr(config, "cudnn_benchmark", False), model=config.model,
                          deterministic=getattr(config, "deterministic", False))
        self.device = set_device(config, self.local_rank)
        self.amp_dtype = torch.float16 if getattr(config, "amp_dtype", "bf16") == "fp16" else torch.bfloat16
        use_scaler = bool(config.amp_training) and self.amp_dtype == torch.float16 and self.device.type == "cuda"
        self.scaler = torch.amp.GradScaler("cuda", enabled=use_scaler)
        if self.main_rank:
            mkdir(config.save_dir)
        set_seed(config.random_seed)
        self.model = get_model(config).to(self.device)
        if getattr(config, "channels_last", False) and self.device.type == "cuda":
            self.model = self.model.to(memory_format=torch.channels_last)

        if config.is_testing:
            self.test_loader = get_test_loader(config)
        else:
            self.writer = get_writer(config, self.main_rank)
            self.loss_fn = get_loss_fn(config, self.device)
            self.train_loader, self.val_loader = get_loader(config, self.local_rank)
            self.optimizer = get_optimizer(config, self.model)
            self.scheduler = get_scheduler(config, self.optimizer, len(self.train_loader))
            self.best_score = 0.0
            self.cur_epoch = 0
            self.train_itrs = 0
        self._resume_state = None
        self.load_ckpt(config)
        if not config.is_testing:
            self.ema_model = get_ema_model(config, self.model, self.device)
            if self._resume_state is not None and self._resume_state.get("ema_state_dict") is not None:
                self.ema_model.ema.load_state_dict(self._resume_state["ema_state_dict"])
            self._resume_state = None
            # fp16 GradScaler may skip a step -> keep the EMA out of the optimizer in that mode
            self.ema_fused = (not self.scaler.is_enabled()) and self.device.type == "cuda" and \
                self.ema_model.attach(self.optimizer, self.model)

    # ------------------------------------------------------------------ run
    def run(self, config):
        self.parallel_model(config)
        if self.main_rank:
            save_config(config)
            log_config(config, self.logger)
        for cur_epoch in range(self.cur_epoch, config.total_epoch):
            self.cur_epoch = cur_epoch
            inject_fault(cur_epoch)
            self.train_one_epoch(config)
            if cur_epoch >= config.begin_val_epoch and cur_epoch % config.val_interval == 0:
                val_score = self.validate(config)
                if self.main_rank and val_score > self.best_score:
                    self.best_score = val_score
                    if config.save_ckpt:
                        self.save_ckpt(config, save_best=True)
            if self.main_rank and config.save_ckpt:
                self.save_ckpt(config)
            barrier()
        if config.use_tb and self.main_rank and self.writer is not None:
            self.writer.flush()
            self.writer.close()
        if config.save_ckpt:
            barrier()
            self.val_best(config)
        destroy_ddp_process(config)

    def parallel_model(self, config):
        self.model = parallel_model(config, self.model, self.local_rank, self.device)

    def train_one_epoch(self, config):
        raise NotImplementedError()

    def validate(self, config, val_best=False):
        raise NotImplementedError()

    def predict(self, config):
        raise NotImplementedError()

    # ------------------------------------------------------------ checkpoint
    def _log(self, msg):
        if self.main_rank and self.logger is not None:
            self.logger.info(msg)

    def load_ckpt(self, config):
        path = config.load_ckpt_path
        if config.load_ckpt and path and os.path.isfile(path):
            ckpt = torch.load(path, map_location=self.device, weights_only=True)
            self.model.load_state_dict(ckpt["state_dict"])
            self._log(f"Load model state dict from {path}")
            if not config.is_testing and config.resume_training:
                self.cur_epoch = int(ckpt["cur_epoch"]) + 1
                self.best_score = ckpt["best_score"]
                if ckpt.get("optimizer") is not None:
                    self.optimizer.load_state_dict(ckpt["optimizer"])
                if ckpt.get("scheduler") is not None:
                    self.scheduler.load_state_dict(ckpt["scheduler"])
                if ckpt.get("scaler") is not None:
                    self.scaler.load_state_dict(ckpt["scaler"])
                self.train_itrs = self.cur_epoch * config.iters_per_epoch
                self._resume_state = {"ema_state_dict": ckpt.get("ema_state_dict")}
                self._log(f"Resume training from {path}")
            del ckpt
        else:
            if config.is_testing:
                raise ValueError(f"Could not find any pretrained checkpoint at path: {path}.")
            self._log("[!] Train from scratch")

    def save_ckpt(self, config, save_best=False):
        if config.ckpt_name is None:
            save_name = "best.pth" if save_best else "last.pth"
        else:
            stem, ext = os.path.splitext(config.ckpt_name)
            save_name = f"{stem}_best{ext or '.pth'}" if save_best else (config.ckpt_name if ext else stem + ".pth")
        path = os.path.join(config.save_dir, save_name)
        state = self.ema_model.ema.state_dict() if save_best else de_parallel(self.model).state_dict()
        payload = {
            "cur_epoch": self.cur_epoch,
            "best_score": self.best_score,
            "state_dict": state,
            "optimizer": None if save_best else self.optimizer.state_dict(),
            "scheduler": None if save_best else self.scheduler.state_dict(),
        }
        if not save_best:
            payload["ema_state_dict"] = self.ema_model.ema.state_dict()
            payload["scaler"] = self.scaler.state_dict() if self.scaler.is_enabled() else None
        tmp = path + ".tmp"
        torch.save(payload, tmp)
        os.replace(tmp, path)  # atomic: a crash never leaves a torn last.pth

    def val_best(self, config, ckpt_path=None):
        ckpt_path = ckpt_path or os.path.join(config.save_dir, "best.pth")
        if not os.path.isfile(ckpt_path):
            raise ValueError(f"Best checkpoint does not exist at {ckpt_path}")
        self._log(f"\nTrain {config.total_epoch} epochs finished!\n")
        self._log(f"{'#' * 50}\nValidation for the best checkpoint...")
        self.model = de_parallel(self.model)
        ckpt = torch.load(ckpt_path, map_location=self.device, weights_only=True)
        self.model.load_state_dict(ckpt["state_dict"])
        del ckpt
        self.ema_model.set_model(self.model)
        val_score = self.validate(config, val_best=True)
        self._log(f"Best validation score is {val_score}.\n")
        return val_score
