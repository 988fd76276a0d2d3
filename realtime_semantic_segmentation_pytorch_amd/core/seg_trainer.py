"""Segmentation trainer (parity: reference core/seg_trainer.py:16-191).

The training step keeps the reference's objective exactly -- main loss + aux
heads (nearest-resized masks, coefficients ``aux_coef``) or the STDC detail
head (Laplacian detail GT, Dice+BCE) + optional Hinton KD -- but is arranged
for the GPU:

* the model runs under bf16 autocast (fp16 + GradScaler when ``amp_dtype='fp16'``)
  on channels-last activations;
* ``defer_final_upsample`` makes the model hand back head-resolution logits and
  the fused HIP loss kernel upsamples inside the loss (no full-resolution
  logits in HBM); aux losses read nearest-resized labels in-kernel;
* there is no host synchronisation inside a step: the loss is only copied to
  the host every ``log_interval`` iterations (the reference syncs >= 5x/step).
"""
from __future__ import annotations

import os

import numpy as np
import torch
from PIL import Image

from .. import ops
from ..models import get_teacher_model
from ..parallel import de_parallel
from ..utils import get_colormap, get_seg_metrics, sampler_set_epoch
from .base_trainer import BaseTrainer
from .loss import kd_loss_fn


class SegTrainer(BaseTrainer):
    def __init__(self, config):
        super().__init__(config)
        self.config = config
        if config.is_testing:
            self.colormap = torch.tensor(get_colormap(config), dtype=torch.uint8, device=self.device)
        else:
            self.teacher_model = get_teacher_model(config, self.device)
            if self.teacher_model is not None and getattr(config, "channels_last", False) and self.device.type == "cuda":
                self.teacher_model = self.teacher_model.to(memory_format=torch.channels_last)
            self.metrics = get_seg_metrics(config).to(self.device)
            if config.use_detail_head:
                from ..models.stdc import LaplacianConv
                from .loss import get_detail_loss_fn

                self.laplacian_conv = LaplacianConv(self.device)
                self.detail_loss_fn = get_detail_loss_fn(config)

    # ------------------------------------------------------------------ step
    def _autocast(self):
        cfg = self.config
        return torch.autocast(device_type=self.device.type, dtype=self.amp_dtype,
                              enabled=bool(cfg.amp_training))

    def _prep(self, images, masks):
        images = images.to(self.device, dtype=torch.float32, non_blocking=True)
        if getattr(self.config, "channels_last", False) and self.device.type == "cuda":
            images = images.contiguous(memory_format=torch.channels_last)
        masks = masks.to(self.device, dtype=torch.long, non_blocking=True)
        return images, masks

    def _gpu_augment(self, img, msk, params):
        """Raw uint8 batch from a ``gpu_aug`` dataset -> augmented (images, masks) on the device."""
        ds = self.train_loader.dataset
        cl = bool(getattr(self.config, "channels_last", False)) and self.device.type == "cuda"
        img = img.to(self.device, non_blocking=True)
        msk = msk.to(self.device, non_blocking=True)
        return ops.augment_batch(img, msk, params, ds.aug_lut, ds.aug_spec, channels_last=cl)

    def _teacher_forward(self, images):
        """Frozen KD teacher.  On the GPU it runs as a captured HIP graph with its weights cast to
        the autocast dtype once (utils/inference.py InferenceEngine): one copy + one graph launch
        per step instead of an eager forward of a few hundred kernels and per-forward weight casts
        (``kd_teacher_graph=False``: eager).  Rebuilt if the batch shape changes."""
        cfg = self.config
        if self.device.type != "cuda" or not getattr(cfg, "kd_teacher_graph", True):
            return self.teacher_model(images)
        key = (tuple(images.shape), images.dtype)
        eng = getattr(self, "_teacher_engine", None)
        if eng is None or eng[0] != key:
            from ..utils.inference import InferenceEngine

            dtype = self.amp_dtype if cfg.amp_training else torch.float32
            with torch.autocast(self.device.type, enabled=False):
                engine = InferenceEngine(self.teacher_model, tuple(images.shape), dtype=dtype,
                                         channels_last=bool(getattr(cfg, "channels_last", False)), warmup=2,
                                         device=self.device)
            self._teacher_engine = eng = (key, engine)
        return eng[1](images)

    def compute_loss(self, images, masks):
        """Forward + total loss. Returns (loss, main_preds, extras dict)."""
        cfg = self.config
        extras = {}
        defer = bool(getattr(cfg, "fused_loss", True))
        # uint8 label maps: the fused loss kernels read them ~4x per step (main/aux x fwd/bwd)
        labels = masks
        if (masks.is_cuda and masks.dtype == torch.int64 and cfg.num_class <= 255
                and 0 <= cfg.ignore_index <= 255):
            labels = masks.to(torch.uint8)
        with self._autocast(), ops.defer_final_upsample(defer):
            if cfg.use_aux:
                preds, preds_aux = self.model(images, is_training=True)
                loss = self.loss_fn(preds, labels)
                if cfg.aux_coef is None:
                    cfg.aux_coef = [1.0] * len(preds_aux)
                coefs = cfg.aux_coef if isinstance(cfg.aux_coef, (list, tuple)) else [cfg.aux_coef]
                if len(coefs) != len(preds_aux):
                    raise ValueError("Auxiliary loss coefficient length does not match.")
                for coef, aux in zip(coefs, preds_aux):
                    loss = loss + float(coef) * self.loss_fn.aux(aux, labels)
            elif cfg.use_detail_head:
                # Laplacian detail target + x8 bilinear resize + Dice + BCE: one fused HIP op
                # (ops/detail.py; the reference formulation on CPU)
                preds, preds_detail = self.model(images, is_training=True)
                loss_detail = ops.detail_loss(preds_detail, labels, de_parallel(self.model).detail_conv,
                                              cfg.detail_thrs, cfg.dice_loss_coef, cfg.bce_loss_coef,
                                              laplacian=self.laplacian_conv)
                loss = self.loss_fn(preds, labels) + cfg.detail_loss_coef * loss_detail
                extras["loss_detail"] = loss_detail
            else:
                preds = self.model(images)
                loss = self.loss_fn(preds, labels)
            if cfg.kd_training:
                with torch.no_grad(), ops.defer_final_upsample(False):
                    teacher_preds = self._teacher_forward(images)
                loss_kd = kd_loss_fn(cfg, preds, teacher_preds)
                extras["loss_main"] = loss
                loss = loss + cfg.kd_loss_coefficient * loss_kd
                extras["loss_kd"] = loss_kd
        return loss, preds, extras

    def _graph_step_ok(self, images):
        cfg = self.config
        return (bool(getattr(cfg, "graph_step", False)) and images.is_cuda and not cfg.DDP
                and not cfg.kd_training and not self.scaler.is_enabled())

    def _graphed_forward_backward(self, images, masks):
        """Forward + loss + backward replayed from ONE captured HIP graph (``graph_step``).

        Small per-GPU batches are launch-bound: a training step is ~900 kernels, each paying the
        host's launch cost.  After ``graph_warmup`` eager steps (per-shape kernel autotune, MIOpen
        find, optimizer state) the forward, the loss and the backward -- including the zeroing of
        the persistent gradient buffers -- are captured once per input shape; a step is then two
        input copies, one graph launch and the (eager, single-launch) fused optimizer, whose
        per-step learning rate / EMA weight therefore stay live.  Non-DDP, non-KD, no GradScaler.
        Returns None while warming up (the caller runs the eager step)."""
        key = (tuple(images.shape), images.dtype, tuple(masks.shape), masks.dtype)
        st = getattr(self, "_gstep", None)
        if st is None or st["key"] != key:
            st = self._gstep = {"key": key, "seen": 0, "graph": None}
        if st["graph"] is None:
            st["seen"] += 1
            if st["seen"] <= int(getattr(self.config, "graph_warmup", 3)):
                return None
            # persistent gradient buffers the graph writes in place: exactly the parameters the
            # last eager step gave a gradient -- a built-but-unused head (aux / detail off) keeps
            # grad None, so the optimizer skips it exactly as in eager training (no weight decay,
            # momentum or Adam-moment updates on a zero gradient)
            grads = [p.grad for p in self.model.parameters() if p.requires_grad and p.grad is not None]
            sx, sy = images.clone(), masks.clone()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                torch._foreach_zero_(grads)
                loss, _, extras = self.compute_loss(sx, sy)
                loss.backward()
            st.update(graph=g, x=sx, y=sy, loss=loss, extras=extras)
        st["x"].copy_(images, non_blocking=True)
        st["y"].copy_(masks, non_blocking=True)
        st["graph"].replay()
        return st["loss"], st["extras"]

    def train_step(self, images, masks):
        done = self._graphed_forward_backward(images, masks) if self._graph_step_ok(images) else None
        if done is not None:
            loss, extras = done
        else:
            if getattr(self, "_gstep", None) is None or self._gstep.get("graph") is None:
                self.optimizer.zero_grad(set_to_none=True)
            else:  # a shape change after capture: keep the graph's gradient buffers
                self.optimizer.zero_grad(set_to_none=False)
            loss, _, extras = self.compute_loss(images, masks)
            self.scaler.scale(loss).backward()
        if self.ema_fused:  # the fused optimizer writes the parameter EMAs in its own launch
            self.optimizer.ema_weight = 1.0 - self.ema_model.decay(self.train_itrs + 1)
        self.scaler.step(self.optimizer)
        self.scaler.update()
        total = getattr(self.scheduler, "total_steps", None)
        if total is None or self.scheduler.last_epoch < total:  # never step OneCycle past its end
            self.scheduler.step()
        self.train_itrs += 1
        self.ema_model.update(self.model, self.train_itrs,
                              params_done=self.ema_fused and getattr(self.optimizer, "last_step_fused", False))
        return loss.detach(), extras

    # ----------------------------------------------------------------- epoch
    def train_one_epoch(self, config):
        self.model.train()
        sampler_set_epoch(config, self.train_loader, self.cur_epoch)
        log_every = max(1, int(getattr(config, "log_interval", 20)))
        max_itrs = getattr(config, "max_train_itrs", None)
        for cur_itrs, batch in enumerate(self.train_loader):
            if max_itrs is not None and cur_itrs >= max_itrs:
                break
            self.cur_itrs = cur_itrs
            images, masks = self._gpu_augment(*batch) if len(batch) == 3 else self._prep(*batch)
            loss, extras = self.train_step(images, masks)
            if self.main_rank and (cur_itrs % log_every == 0):
                lv = float(loss)
                if config.use_tb and self.writer is not None:
                    self.writer.add_scalar("train/loss", lv, self.train_itrs)
                    if "loss_detail" in extras:
                        self.writer.add_scalar("train/loss_detail", float(extras["loss_detail"]), self.train_itrs)
                    if "loss_kd" in extras:
                        self.writer.add_scalar("train/loss_kd", float(extras["loss_kd"]), self.train_itrs)
                        self.writer.add_scalar("train/loss_total", lv, self.train_itrs)
                if self.logger is not None:
                    self.logger.info(f"Epoch:{self.cur_epoch}/{config.total_epoch}    | "
                                     f"Itr:{cur_itrs}/{len(self.train_loader)}    | Loss:{lv:4.4g}")

    @torch.no_grad()
    def validate(self, config, val_best=False):
        model = self.ema_model.ema
        model.eval()
        for images, masks in self.val_loader:
            images, masks = self._prep(images, masks)
            with self._autocast():
                preds = model(images)
            self.metrics.update(preds, masks)
        iou = self.metrics.compute()
        score = float(iou.mean())
        if self.main_rank:
            if val_best:
                self._log(f"\n\nTrain {config.total_epoch} epochs finished.\n\nBest mIoU is: {score:.4f}\n")
            else:
                self._log(f" Epoch{self.cur_epoch} mIoU: {score:.4f}    | best mIoU so far: {self.best_score:.4f}\n")
            if config.use_tb and self.writer is not None and self.cur_epoch < config.total_epoch and not val_best:
                self.writer.add_scalar("val/mIoU", score, self.cur_epoch + 1)
                for i in range(config.num_class):
                    self.writer.add_scalar(f"val/IoU_cls{i:02d}", float(iou[i]), self.cur_epoch + 1)
        self.metrics.reset()
        return score

    @torch.no_grad()
    def predict(self, config):
        if config.DDP:
            raise ValueError("Predict mode currently does not support DDP.")
        self._log("\nStart predicting...\n")
        out_dir = os.path.join(config.save_dir, "predicts")
        os.makedirs(out_dir, exist_ok=True)
        self.model.eval()
        for images, images_aug, names in self.test_loader:
            images_aug = images_aug.to(self.device, dtype=torch.float32)
            if getattr(config, "channels_last", False) and self.device.type == "cuda":
                images_aug = images_aug.contiguous(memory_format=torch.channels_last)
            with self._autocast():
                preds = self.model(images_aug)
            logits = ops.materialize(preds)
            raws = [np.asarray(im).astype(np.uint8) for im in images] if config.blend_prediction else None
            # argmax + colormap (+ blend when the raw images match the logits' size) in one kernel
            same = raws is not None and all(r.shape == (*logits.shape[2:], 3) for r in raws)
            raw_dev = torch.from_numpy(np.stack(raws)).to(self.device) if same else None
            _, colored, blended = ops.colorize(logits, self.colormap, raw_dev, config.blend_alpha)
            colored = colored.cpu().numpy()
            blended = blended.cpu().numpy() if blended is not None else None
            for i, name in enumerate(names):
                path = os.path.join(out_dir, name)
                suffix = name.rsplit(".", 1)[-1] if "." in name else "png"
                mask_img = Image.fromarray(colored[i])
                if config.save_mask:
                    mask_img.save(path)
                if config.blend_prediction:
                    if blended is not None:
                        out = Image.fromarray(blended[i])
                    else:
                        raw = Image.fromarray(raws[i])
                        if raw.size != mask_img.size:
                            raw = raw.resize(mask_img.size, Image.BILINEAR)
                        out = Image.blend(raw, mask_img, config.blend_alpha)
                    out.save(path[: -len(suffix) - 1] + f"_blend.{suffix}" if "." in name else path + "_blend.png")
