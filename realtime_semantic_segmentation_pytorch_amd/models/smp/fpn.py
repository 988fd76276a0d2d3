"""FPN decoder (SMP layout): top-down pyramid (nearest x2 + 1x1 lateral), per-level
3x3 Conv-GroupNorm-ReLU towers upsampled to 1/4, merged by add or concat.

Behavioural target: SMP ``FPN`` (reference models/__init__.py:42-44).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import ops
from .base import SegmentationHead, SegmentationModel
from .encoders import get_encoder


class Conv3x3GNReLU(nn.Module):
    def __init__(self, in_channels, out_channels, upsample=False):
        super().__init__()
        self.upsample = upsample
        self.block = nn.Sequential(nn.Conv2d(in_channels, out_channels, 3, 1, 1, bias=False),
                                   nn.GroupNorm(32, out_channels), nn.ReLU(inplace=True))

    def forward(self, x):
        x = self.block(x)
        if self.upsample:
            x = ops.interpolate(x, (x.shape[2] * 2, x.shape[3] * 2), True)
        return x


class FPNBlock(nn.Module):
    def __init__(self, pyramid_channels, skip_channels):
        super().__init__()
        self.skip_conv = nn.Conv2d(skip_channels, pyramid_channels, kernel_size=1)

    def forward(self, x, skip=None):
        s = self.skip_conv(skip)
        return F.interpolate(x, scale_factor=2, mode="nearest").to(s.dtype) + s


class SegmentationBlock(nn.Module):
    def __init__(self, in_channels, out_channels, n_upsamples=0):
        super().__init__()
        blocks = [Conv3x3GNReLU(in_channels, out_channels, upsample=bool(n_upsamples))]
        blocks += [Conv3x3GNReLU(out_channels, out_channels, upsample=True) for _ in range(1, n_upsamples)]
        self.block = nn.Sequential(*blocks)

    def forward(self, x):
        return self.block(x)


class MergeBlock(nn.Module):
    def __init__(self, policy):
        super().__init__()
        if policy not in ("add", "cat"):
            raise ValueError(f"`merge_policy` must be one of: ['add', 'cat'], got {policy}")
        self.policy = policy

    def forward(self, x):
        if self.policy == "add":
            out = x[0]
            for t in x[1:]:
                out = out + t
            return out
        return torch.cat(x, dim=1)


class FPNDecoder(nn.Module):
    def __init__(self, encoder_channels, encoder_depth=5, pyramid_channels=256, segmentation_channels=128,
                 dropout=0.2, merge_policy="add"):
        super().__init__()
        self.out_channels = segmentation_channels if merge_policy == "add" else segmentation_channels * 4
        if encoder_depth < 3:
            raise ValueError(f"Encoder depth for FPN decoder cannot be less than 3, got {encoder_depth}.")
        enc = list(encoder_channels)[::-1][: encoder_depth + 1]
        self.p5 = nn.Conv2d(enc[0], pyramid_channels, kernel_size=1)
        self.p4 = FPNBlock(pyramid_channels, enc[1])
        self.p3 = FPNBlock(pyramid_channels, enc[2])
        self.p2 = FPNBlock(pyramid_channels, enc[3])
        self.seg_blocks = nn.ModuleList([SegmentationBlock(pyramid_channels, segmentation_channels, n)
                                         for n in (3, 2, 1, 0)])
        self.merge = MergeBlock(merge_policy)
        self.dropout = nn.Dropout2d(p=dropout, inplace=True)

    def forward(self, *features):
        c2, c3, c4, c5 = features[-4:]
        p5 = self.p5(c5)
        p4 = self.p4(p5, c4)
        p3 = self.p3(p4, c3)
        p2 = self.p2(p3, c2)
        x = self.merge([blk(p) for blk, p in zip(self.seg_blocks, (p5, p4, p3, p2))])
        return self.dropout(x)


class FPN(SegmentationModel):
    def __init__(self, encoder_name="resnet34", encoder_depth=5, encoder_weights="imagenet",
                 decoder_pyramid_channels=256, decoder_segmentation_channels=128, decoder_merge_policy="add",
                 decoder_dropout=0.2, in_channels=3, classes=1, upsampling=4):
        super().__init__()
        self.encoder = get_encoder(encoder_name, in_channels, encoder_depth, encoder_weights)
        self.decoder = FPNDecoder(self.encoder.out_channels, encoder_depth, decoder_pyramid_channels,
                                  decoder_segmentation_channels, decoder_dropout, decoder_merge_policy)
        self.segmentation_head = SegmentationHead(self.decoder.out_channels, classes, kernel_size=1,
                                                  upsampling=upsampling)
        self.initialize()
