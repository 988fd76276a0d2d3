"""Cityscapes fine annotations (parity: reference datasets/cityscapes.py:11-162).

Layout: ``{data_root}/leftImg8bit/{mode}/{city}/*_leftImg8bit.png`` and
``{data_root}/gtFine/{mode}/{city}/*_gtFine_labelIds.png``.  Masks are mapped
from label ids to the 19 train ids (255 = ignore) AFTER augmentation, so pad
value 0 ('unlabeled') becomes ignore exactly like the reference.
"""
from __future__ import annotations

import os

import numpy as np
import torch
from PIL import Image
from torch.utils.data import Dataset

from . import transforms as T

# label id -> train id for ids 0..33 (+ 'license plate' id -1 stored last), from
# the official cityscapesScripts label table.
_TRAIN_IDS = [255, 255, 255, 255, 255, 255, 255, 0, 1, 255, 255, 2, 3, 4, 255, 255, 255, 5, 255,
              6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 255, 255, 16, 17, 18, -1]
CLASS_NAMES = ["road", "sidewalk", "building", "wall", "fence", "pole", "traffic light",
               "traffic sign", "vegetation", "terrain", "sky", "person", "rider", "car", "truck",
               "bus", "train", "motorcycle", "bicycle"]


def split_key(key):
    """Dataset key -> (index, epoch): ``EpochSampler`` yields (index, epoch) pairs, plain
    samplers (and direct ``ds[i]``) yield the index alone (epoch 0)."""
    if isinstance(key, (tuple, list)):
        return int(key[0]), int(key[1])
    return int(key), 0


def sample_rng(seed: int, epoch: int, index: int) -> np.random.Generator:
    """Augmentation stream of one (epoch, sample) draw.

    The reference's albumentations pipeline draws fresh randomness on every call
    (reference datasets/cityscapes.py:115-124).  Seeding from (seed, epoch, index) keeps that
    -- a sample gets a new scale / crop / jitter / flip every epoch -- while staying
    reproducible and independent of the worker count or persistent workers (the epoch comes
    from the sampler, in the main process)."""
    return np.random.default_rng([int(seed) % (2 ** 63), int(epoch), int(index)])


def aug_spec(transform):
    """Static crop / pad / normalisation of a training pipeline (for ops.augment_batch)."""
    from ..ops.augment import draw_params

    big = 1 << 15  # any source larger than the crop: the spec does not depend on the draws
    return draw_params(transform, big, big, np.random.default_rng(0))[1]


def raw_sample(transform, image, mask, rng):
    """GPU-augmentation sample: (uint8 [H, W, 3] image, uint8 [H, W] raw labels, fp32 params)
    with the parameters drawn from ``rng`` exactly as ``transform`` would draw them."""
    from ..ops.augment import draw_params

    params, _ = draw_params(transform, image.shape[0], image.shape[1], rng)
    return (torch.from_numpy(np.require(image, np.uint8, ["C", "W"])),
            torch.from_numpy(np.require(mask, np.uint8, ["C", "W"])), torch.from_numpy(params))


class Cityscapes(Dataset):
    id_to_train_id = np.array(_TRAIN_IDS)
    # uint8 lookup (255 for anything unknown) used by encode_target
    _lut = np.full(256, 255, np.uint8)
    _lut[:34] = np.array(_TRAIN_IDS[:34], np.int64).clip(0, 255).astype(np.uint8)

    def __init__(self, config, mode="train"):
        root = os.path.expanduser(config.data_root or config.dataroot or "")
        img_dir = os.path.join(root, "leftImg8bit", mode)
        msk_dir = os.path.join(root, "gtFine", mode)
        if not os.path.isdir(img_dir):
            raise RuntimeError(f"Image directory: {img_dir} does not exist.")
        if not os.path.isdir(msk_dir):
            raise RuntimeError(f"Mask directory: {msk_dir} does not exist.")
        self.mode = mode
        self.seed = int(getattr(config, "random_seed", 1))
        self.transform = T.train_transform(config) if mode == "train" else T.val_transform(config)
        # GPU augmentation (ops/augment.py): __getitem__ returns the decoded raw image and label
        # ids plus the drawn parameters; the trainer runs the pixel work on the device
        self.gpu_aug = mode == "train" and bool(getattr(config, "gpu_aug", False))
        self.aug_lut = torch.from_numpy(self._lut.copy())
        self.aug_spec = aug_spec(self.transform) if self.gpu_aug else None
        self.images, self.masks = [], []
        for city in sorted(os.listdir(img_dir)):
            for name in sorted(os.listdir(os.path.join(img_dir, city))):
                self.images.append(os.path.join(img_dir, city, name))
                stem = name.split("_leftImg8bit")[0]
                self.masks.append(os.path.join(msk_dir, city, f"{stem}_gtFine_labelIds.png"))

    def __len__(self):
        return len(self.images)

    def __getitem__(self, key):
        index, epoch = split_key(key)
        image = np.asarray(Image.open(self.images[index]).convert("RGB"))
        mask = np.asarray(Image.open(self.masks[index]).convert("L"))
        if self.gpu_aug:
            return raw_sample(self.transform, image, mask, sample_rng(self.seed, epoch, index))
        image, mask = self.transform(image, mask, sample_rng(self.seed, epoch, index))
        return T.to_tensor(image), torch.from_numpy(self.encode_target(mask).astype(np.int64))

    @classmethod
    def encode_target(cls, mask):
        return cls._lut[np.asarray(mask, dtype=np.uint8)]
