"""Logging / seeding / config dump / colormaps (parity: reference utils/utils.py:5-78).

The reference uses loguru + TensorBoard (not installed here).  This module uses
stdlib ``logging`` with the reference's ``[YYYY-MM-DD HH:mm] msg`` format, and a
TensorBoard ``SummaryWriter`` when ``tensorboard`` is importable, otherwise a
JSON-lines scalar writer with the same ``add_scalar/flush/close`` surface.
"""
from __future__ import annotations

import json
import logging
import os
import random
import sys
import time

import numpy as np
import torch


def mkdir(path):
    if path:
        os.makedirs(path, exist_ok=True)


def set_seed(seed):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


class JsonlWriter:
    """Minimal scalar writer: one JSON object per ``add_scalar`` call."""

    def __init__(self, log_dir):
        mkdir(log_dir)
        self.path = os.path.join(log_dir, "scalars.jsonl")
        self._f = open(self.path, "a", buffering=1)

    def add_scalar(self, tag, value, step):
        if torch.is_tensor(value):
            value = value.detach().float().item()
        self._f.write(json.dumps({"tag": tag, "value": float(value), "step": int(step),
                                  "time": time.time()}) + "\n")

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


def get_writer(config, main_rank):
    if not (config.use_tb and main_rank):
        return None
    try:
        from torch.utils.tensorboard import SummaryWriter  # noqa: F401

        return SummaryWriter(config.tb_log_dir)
    except Exception:
        return JsonlWriter(config.tb_log_dir)


def get_logger(config, main_rank):
    if not main_rank:
        return None
    name = getattr(config, "logger_name", "seg_trainer")
    logger = logging.getLogger(f"rtseg.{name}.{id(config)}")
    if logger.handlers:
        return logger
    logger.setLevel(logging.INFO)
    logger.propagate = False
    fmt = logging.Formatter("[%(asctime)s] %(message)s", datefmt="%Y-%m-%d %H:%M")
    sh = logging.StreamHandler(sys.stderr)
    sh.setFormatter(fmt)
    logger.addHandler(sh)
    mkdir(config.save_dir)
    fh = logging.FileHandler(os.path.join(config.save_dir, f"{name}.log"))
    fh.setFormatter(fmt)
    logger.addHandler(fh)
    return logger


def _jsonable(v):
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if torch.is_tensor(v):
        return v.tolist()
    return str(v)


def save_config(config):
    mkdir(config.save_dir)
    with open(os.path.join(config.save_dir, "config.json"), "w") as f:
        json.dump({k: _jsonable(v) for k, v in vars(config).items()}, f, indent=4)


_SUMMARY_KEYS = ["dataset", "num_class", "model", "encoder", "decoder", "arch_type", "loss_type",
                 "optimizer_type", "lr_policy", "total_epoch", "train_bs", "val_bs", "train_num",
                 "val_num", "gpu_num", "num_workers", "amp_training", "amp_dtype", "DDP",
                 "kd_training", "use_ema", "use_aux", "use_detail_head", "channels_last"]


def log_config(config, logger):
    if logger is None:
        return
    lines = [f"{'#' * 25} Config Informations {'#' * 25}"]
    for k in _SUMMARY_KEYS:
        if hasattr(config, k):
            lines.append(f"{k}: {getattr(config, k)}")
    lines.append("#" * 71)
    logger.info("\n".join(lines))


CITYSCAPES_COLORS = [
    (128, 64, 128), (244, 35, 232), (70, 70, 70), (102, 102, 156), (190, 153, 153),
    (153, 153, 153), (250, 170, 30), (220, 220, 0), (107, 142, 35), (152, 251, 152),
    (70, 130, 180), (220, 20, 60), (255, 0, 0), (0, 0, 142), (0, 0, 70), (0, 60, 100),
    (0, 80, 100), (0, 0, 230), (119, 11, 32),
]


def get_colormap(config):
    if config.colormap == "cityscapes":
        return [list(c) for c in CITYSCAPES_COLORS]
    if config.colormap == "custom":
        # deterministic distinct colours for any class count (reference raises here)
        rng = np.random.RandomState(0)
        return rng.randint(0, 255, size=(max(config.num_class, 1), 3)).tolist()
    raise NotImplementedError(f"Unsupport colormap type: {config.colormap}")
