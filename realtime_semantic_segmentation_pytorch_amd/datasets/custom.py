"""Custom dataset produced by ``tools/check_datasets.py`` (parity: reference datasets/custom.py:12-84).

``{data_root}/data.yaml`` holds ``path`` and ``names``; images/masks live in
``{path}/{mode}/{imgs,masks}`` with identical stems (masks ``.png``, values =
class ids).  Images are scaled to [0, 1] (mean 0 / std 1 like the reference).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import yaml
from PIL import Image
from torch.utils.data import Dataset

from . import transforms as T
from .cityscapes import aug_spec, raw_sample, sample_rng, split_key


class Custom(Dataset):
    def __init__(self, config, mode="train"):
        root = os.path.expanduser(config.data_root or config.dataroot or "")
        cfg_path = os.path.join(root, "data.yaml")
        if not os.path.exists(cfg_path):
            raise FileNotFoundError(f"{cfg_path} not exists.")
        with open(cfg_path, "r", encoding="utf-8") as f:
            meta = yaml.safe_load(f)
        base = meta.get("path", root)
        names = meta["names"]
        self.class_names = [names[k] for k in sorted(names)] if isinstance(names, dict) else list(names)
        self.id_to_train_id = {i: i for i in range(len(self.class_names))}
        img_dir = os.path.join(base, mode, "imgs")
        msk_dir = os.path.join(base, mode, "masks")
        if not os.path.isdir(img_dir):
            raise RuntimeError(f"Image directory: {img_dir} does not exist.")
        if not os.path.isdir(msk_dir):
            raise RuntimeError(f"Mask directory: {msk_dir} does not exist.")
        self.seed = int(getattr(config, "random_seed", 1))
        norm = ((0.0, 0.0, 0.0), (1.0, 1.0, 1.0))
        if mode == "train":
            self.transform = T.train_transform(config, norm, square_size=config.train_size)
        else:
            self.transform = T.val_transform(config, norm, square_size=config.test_size)
        # GPU augmentation needs one source size per batch: not with ResizeToSquare (train_size)
        self.gpu_aug = mode == "train" and bool(getattr(config, "gpu_aug", False))
        if self.gpu_aug and config.train_size is not None:
            raise ValueError("gpu_aug does not support train_size (ResizeToSquare); unset one of them")
        self.aug_lut = torch.arange(256, dtype=torch.uint8)  # masks already hold class ids
        self.aug_spec = aug_spec(self.transform) if self.gpu_aug else None
        self.images, self.masks = [], []
        for name in sorted(os.listdir(img_dir)):
            self.images.append(os.path.join(img_dir, name))
            self.masks.append(os.path.join(msk_dir, os.path.splitext(name)[0] + ".png"))

    def __len__(self):
        return len(self.images)

    def __getitem__(self, key):
        index, epoch = split_key(key)
        image = np.asarray(Image.open(self.images[index]).convert("RGB"))
        mask = np.asarray(Image.open(self.masks[index]).convert("L"))
        if self.gpu_aug:
            return raw_sample(self.transform, image, mask, sample_rng(self.seed, epoch, index))
        image, mask = self.transform(image, mask, sample_rng(self.seed, epoch, index))
        return T.to_tensor(image), torch.from_numpy(np.asarray(mask, np.int64))
