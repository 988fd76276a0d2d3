"""LinkNet decoder (SMP layout): 1x1 reduce -> 4x4 stride-2 transposed conv -> 1x1 expand, + skip.

Behavioural target: SMP ``Linknet`` (reference models/__init__.py:42-44).
"""
from __future__ import annotations

import torch.nn as nn

from ... import ops
from .base import Conv2dReLU, SegmentationHead, SegmentationModel
from .encoders import get_encoder


class TransposeX2(nn.Sequential):
    def __init__(self, in_channels, out_channels, use_batchnorm=True):
        layers = [nn.ConvTranspose2d(in_channels, out_channels, kernel_size=4, stride=2, padding=1)]
        if use_batchnorm:
            layers.append(nn.BatchNorm2d(out_channels))
        layers.append(nn.ReLU(inplace=True))
        super().__init__(*layers)

    def forward(self, x):
        y = self[0](x)
        if isinstance(self[1], nn.BatchNorm2d):
            return ops.bn_act(y, self[1], "relu")
        return y.relu()


class DecoderBlock(nn.Module):
    def __init__(self, in_channels, out_channels, use_batchnorm=True):
        super().__init__()
        q = in_channels // 4
        self.block = nn.Sequential(Conv2dReLU(in_channels, q, 1, use_batchnorm=use_batchnorm),
                                   TransposeX2(q, q, use_batchnorm=use_batchnorm),
                                   Conv2dReLU(q, out_channels, 1, use_batchnorm=use_batchnorm))

    def forward(self, x, skip=None):
        y = self.block(x)
        return y if skip is None else y + skip


class LinknetDecoder(nn.Module):
    def __init__(self, encoder_channels, prefinal_channels=32, n_blocks=5, use_batchnorm=True):
        super().__init__()
        ch = list(encoder_channels[1:])[::-1] + [prefinal_channels]
        self.blocks = nn.ModuleList([DecoderBlock(ch[i], ch[i + 1], use_batchnorm) for i in range(n_blocks)])

    def forward(self, *features):
        feats = list(features[1:])[::-1]
        x, skips = feats[0], feats[1:]
        for i, blk in enumerate(self.blocks):
            x = blk(x, skips[i] if i < len(skips) else None)
        return x


class Linknet(SegmentationModel):
    def __init__(self, encoder_name="resnet34", encoder_depth=5, encoder_weights="imagenet", decoder_use_batchnorm=True,
                 in_channels=3, classes=1):
        super().__init__()
        self.encoder = get_encoder(encoder_name, in_channels, encoder_depth, encoder_weights)
        self.decoder = LinknetDecoder(self.encoder.out_channels, 32, encoder_depth, decoder_use_batchnorm)
        self.segmentation_head = SegmentationHead(32, classes, kernel_size=1)
        self.initialize()
