"""Inference image folder (parity: reference datasets/test_dataset.py:10-40).

Returns ``(raw uint8 HxWx3, normalised CHW float tensor, file name)``.
"""
from __future__ import annotations

import os

import numpy as np
from PIL import Image
from torch.utils.data import Dataset

from . import transforms as T


class TestDataset(Dataset):
    def __init__(self, config):
        folder = os.path.expanduser(config.test_data_folder or "")
        if not os.path.isdir(folder):
            raise RuntimeError(f"Test image directory: {folder} does not exist.")
        self.transform = T.Compose([T.Scale(config.scale), T.Normalize()])
        self.img_names = sorted(os.listdir(folder))
        self.images = [os.path.join(folder, n) for n in self.img_names]

    def __len__(self):
        return len(self.images)

    def __getitem__(self, index):
        image = np.asarray(Image.open(self.images[index]).convert("RGB"))
        aug, _ = self.transform(image, None)
        return image, T.to_tensor(aug), self.img_names[index]
