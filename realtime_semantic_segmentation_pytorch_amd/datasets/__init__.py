"""Dataset / loader factory (parity: reference datasets/__init__.py:5-64).

Fixes vs the reference: the DistributedSampler uses the
GLOBAL rank (multi-node correct) and ``num_workers`` is per rank.
``config.synthetic_data=True`` swaps in synthetic Cityscapes-shaped data.
"""
from __future__ import annotations

import torch
from torch.utils.data import DataLoader, RandomSampler, Sampler

from .cityscapes import Cityscapes
from .custom import Custom
from .synthetic import DeviceBatches, SyntheticSegDataset
from .test_dataset import TestDataset

dataset_hub = {"cityscapes": Cityscapes, "custom": Custom}


def get_dataset(config):
    if getattr(config, "synthetic_data", False):
        size = config.synthetic_size or (config.crop_h, config.crop_w)
        n = int(config.synthetic_len)
        learn = bool(getattr(config, "synthetic_learnable", False))
        cell = int(getattr(config, "synthetic_cell", 32))
        return (SyntheticSegDataset(n, size, config.num_class, config.ignore_index, seed=0, learnable=learn, cell=cell),
                SyntheticSegDataset(max(1, n // 4), size, config.num_class, config.ignore_index, seed=1,
                                    learnable=learn, cell=cell))
    if config.dataset not in dataset_hub:
        raise NotImplementedError("Unsupported dataset!")
    cls = dataset_hub[config.dataset]
    return cls(config=config, mode="train"), cls(config=config, mode="val")


class EpochSampler(Sampler):
    """Wraps a sampler so it yields ``(index, epoch)``: the datasets seed their augmentation
    from (random_seed, epoch, index), so every epoch draws new augmentations, reproducibly and
    independently of worker processes (persistent workers never see a ``set_epoch``; the keys
    they receive carry it)."""

    def __init__(self, base: Sampler):
        self.base = base
        self.epoch = 0

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)
        if hasattr(self.base, "set_epoch"):
            self.base.set_epoch(epoch)

    def __iter__(self):
        e = self.epoch
        return ((int(i), e) for i in self.base)

    def __len__(self):
        return len(self.base)


def get_loader(config, rank=None, pin_memory=True):
    train_ds, val_ds = get_dataset(config)
    config.train_num = int(len(train_ds) // config.train_bs * config.train_bs)
    config.val_num = len(val_ds)
    workers = int(getattr(config, "num_workers", 0))
    pin = pin_memory and torch.cuda.is_available()
    persistent = workers > 0
    if config.DDP:
        from torch.utils.data.distributed import DistributedSampler

        grank = config.global_rank if getattr(config, "global_rank", None) is not None else (rank or 0)
        tr_s = DistributedSampler(train_ds, num_replicas=config.gpu_num, rank=grank, shuffle=True,
                                  seed=config.random_seed, drop_last=True)
        va_s = DistributedSampler(val_ds, num_replicas=config.gpu_num, rank=grank, shuffle=False)
        train_loader = DataLoader(train_ds, batch_size=config.train_bs, sampler=EpochSampler(tr_s),
                                  num_workers=workers, pin_memory=pin, drop_last=True,
                                  persistent_workers=persistent)
        val_loader = DataLoader(val_ds, batch_size=config.val_bs, sampler=va_s, num_workers=workers,
                                pin_memory=pin, persistent_workers=persistent)
    else:
        gen = torch.Generator().manual_seed(int(config.random_seed))
        train_loader = DataLoader(train_ds, batch_size=config.train_bs,
                                  sampler=EpochSampler(RandomSampler(train_ds, generator=gen)),
                                  num_workers=workers, pin_memory=pin, drop_last=True,
                                  persistent_workers=persistent)
        val_loader = DataLoader(val_ds, batch_size=config.val_bs, shuffle=False,
                                num_workers=workers, pin_memory=pin, persistent_workers=persistent)
    return train_loader, val_loader


def _collate_test(batch):
    raws, tens, names = zip(*batch)
    return list(raws), torch.stack(tens), list(names)


def get_test_loader(config):
    ds = TestDataset(config)
    config.test_num = len(ds)
    if config.DDP:
        raise NotImplementedError("Predict mode does not support DDP.")
    # images of different sizes cannot be stacked: fall back to batch 1 then
    return DataLoader(ds, batch_size=config.test_bs, shuffle=False,
                      num_workers=int(getattr(config, "num_workers", 0)), collate_fn=_collate_test)


__all__ = ["EpochSampler", "Cityscapes", "Custom", "TestDataset", "SyntheticSegDataset", "DeviceBatches",
           "get_dataset", "get_loader", "get_test_loader", "dataset_hub"]
