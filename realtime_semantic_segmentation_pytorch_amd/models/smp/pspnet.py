"""PSPNet decoder (SMP layout): pyramid pooling (1, 2, 3, 6) on the depth-3 (1/8) encoder feature.

Behavioural target: SMP ``PSPNet`` (reference models/__init__.py:42-44): the
encoder is truncated to depth 3, the 1x1 pooling branch has no BatchNorm,
the head is a 3x3 conv with x8 bilinear upsampling.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ... import ops
from .base import Conv2dReLU, SegmentationHead, SegmentationModel
from .encoders import get_encoder


class PSPBlock(nn.Module):
    def __init__(self, in_channels, out_channels, pool_size, use_bathcnorm=True):
        super().__init__()
        if pool_size == 1:
            use_bathcnorm = False  # BatchNorm over a 1x1 map per sample is degenerate
        self.pool = nn.Sequential(nn.AdaptiveAvgPool2d((pool_size, pool_size)),
                                  Conv2dReLU(in_channels, out_channels, (1, 1), use_batchnorm=use_bathcnorm))

    def forward(self, x):
        return ops.interpolate(self.pool(x), x.shape[2:], True)


class PSPModule(nn.Module):
    def __init__(self, in_channels, sizes=(1, 2, 3, 6), use_bathcnorm=True):
        super().__init__()
        self.blocks = nn.ModuleList([PSPBlock(in_channels, in_channels // len(sizes), s, use_bathcnorm)
                                     for s in sizes])

    def forward(self, x):
        feats = [blk(x) for blk in self.blocks]
        return torch.cat([f.to(x.dtype) for f in feats] + [x], dim=1)


class PSPDecoder(nn.Module):
    def __init__(self, encoder_channels, use_batchnorm=True, out_channels=512, dropout=0.2):
        super().__init__()
        self.psp = PSPModule(encoder_channels[-1], (1, 2, 3, 6), use_batchnorm)
        self.conv = Conv2dReLU(encoder_channels[-1] * 2, out_channels, 1, use_batchnorm=use_batchnorm)
        self.dropout = nn.Dropout2d(p=dropout)

    def forward(self, *features):
        return self.dropout(self.conv(self.psp(features[-1])))


class PSPNet(SegmentationModel):
    def __init__(self, encoder_name="resnet34", encoder_weights="imagenet", encoder_depth=3, psp_out_channels=512,
                 psp_use_batchnorm=True, psp_dropout=0.2, in_channels=3, classes=1, upsampling=8):
        super().__init__()
        self.encoder = get_encoder(encoder_name, in_channels, encoder_depth, encoder_weights)
        self.decoder = PSPDecoder(self.encoder.out_channels, psp_use_batchnorm, psp_out_channels, psp_dropout)
        self.segmentation_head = SegmentationHead(psp_out_channels, classes, kernel_size=3, upsampling=upsampling)
        self.initialize()
