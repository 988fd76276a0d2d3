"""U-Net and U-Net++ decoders (SMP layout).

Behavioural target: SMP ``Unet`` / ``UnetPlusPlus`` (reference
models/__init__.py:42-44): nearest x2 upsample, concat skip, two 3x3
Conv2dReLU per block; U-Net++ builds the nested dense skip grid
``x_{depth}_{layer}``.  Head: 3x3 conv at full resolution.

VGG encoders (``encoder_name`` starting with ``vgg``) get SMP's center block: two 3x3 Conv2dReLU
at the deepest feature's width (``decoder.center.{0,1}.*``).  U-Net runs it on the deepest
feature before the first decoder block; U-Net++ builds it (same state-dict keys as SMP) but, as in
SMP, its forward never calls it -- those parameters get no gradient there.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .base import Conv2dReLU, SegmentationHead, SegmentationModel
from .encoders import get_encoder


class CenterBlock(nn.Sequential):
    """SMP's center block of VGG-encoder U-Nets: Conv2dReLU x 2 at ``channels``."""

    def __init__(self, in_channels, out_channels, use_batchnorm=True):
        super().__init__(Conv2dReLU(in_channels, out_channels, 3, padding=1, use_batchnorm=use_batchnorm),
                         Conv2dReLU(out_channels, out_channels, 3, padding=1, use_batchnorm=use_batchnorm))


class DecoderBlock(nn.Module):
    def __init__(self, in_channels, skip_channels, out_channels, use_batchnorm=True, attention_type=None):
        super().__init__()
        if attention_type is not None:
            raise NotImplementedError("decoder_attention_type is not supported")
        self.conv1 = Conv2dReLU(in_channels + skip_channels, out_channels, 3, padding=1, use_batchnorm=use_batchnorm)
        self.attention1 = nn.Identity()
        self.conv2 = Conv2dReLU(out_channels, out_channels, 3, padding=1, use_batchnorm=use_batchnorm)
        self.attention2 = nn.Identity()

    def forward(self, x, skip=None):
        x = F.interpolate(x, scale_factor=2, mode="nearest")
        if skip is not None:
            x = torch.cat([x, skip.to(x.dtype)], dim=1)
        return self.conv2(self.conv1(x))


def _decoder_channels(encoder_channels, decoder_channels):
    enc = list(encoder_channels[1:])[::-1]  # drop the input, start from the deepest feature
    return enc, [enc[0]] + list(decoder_channels[:-1]), enc[1:] + [0], list(decoder_channels)


class UnetDecoder(nn.Module):
    def __init__(self, encoder_channels, decoder_channels, n_blocks=5, use_batchnorm=True, attention_type=None,
                 center=False):
        super().__init__()
        if n_blocks != len(decoder_channels):
            raise ValueError(f"Model depth is {n_blocks}, but you provide `decoder_channels` for "
                             f"{len(decoder_channels)} blocks.")
        enc, ins, skips, outs = _decoder_channels(encoder_channels, decoder_channels)
        self.center = CenterBlock(enc[0], enc[0], use_batchnorm) if center else nn.Identity()
        self.blocks = nn.ModuleList([DecoderBlock(i, s, o, use_batchnorm, attention_type)
                                     for i, s, o in zip(ins, skips, outs)])

    def forward(self, *features):
        feats = list(features[1:])[::-1]
        x, skips = self.center(feats[0]), feats[1:]
        for i, blk in enumerate(self.blocks):
            x = blk(x, skips[i] if i < len(skips) else None)
        return x


class Unet(SegmentationModel):
    def __init__(self, encoder_name="resnet34", encoder_depth=5, encoder_weights="imagenet", decoder_use_batchnorm=True,
                 decoder_channels=(256, 128, 64, 32, 16), decoder_attention_type=None, in_channels=3, classes=1):
        super().__init__()
        self.encoder = get_encoder(encoder_name, in_channels, encoder_depth, encoder_weights)
        self.decoder = UnetDecoder(self.encoder.out_channels, decoder_channels, encoder_depth, decoder_use_batchnorm,
                                   decoder_attention_type, center=encoder_name.startswith("vgg"))
        self.segmentation_head = SegmentationHead(decoder_channels[-1], classes, kernel_size=3)
        self.initialize()


class UnetPlusPlusDecoder(nn.Module):
    def __init__(self, encoder_channels, decoder_channels, n_blocks=5, use_batchnorm=True, attention_type=None,
                 center=False):
        super().__init__()
        if n_blocks != len(decoder_channels):
            raise ValueError(f"Model depth is {n_blocks}, but you provide `decoder_channels` for "
                             f"{len(decoder_channels)} blocks.")
        enc, self.in_channels, self.skip_channels, self.out_channels = _decoder_channels(encoder_channels,
                                                                                          decoder_channels)
        # built for the state-dict layout; unused by forward, as in SMP
        self.center = CenterBlock(enc[0], enc[0], use_batchnorm) if center else nn.Identity()
        blocks = {}
        for layer in range(len(self.in_channels) - 1):
            for depth in range(layer + 1):
                if depth == 0:
                    in_ch = self.in_channels[layer]
                    skip_ch = self.skip_channels[layer] * (layer + 1)
                    out_ch = self.out_channels[layer]
                else:
                    out_ch = self.skip_channels[layer]
                    skip_ch = self.skip_channels[layer] * (layer + 1 - depth)
                    in_ch = self.skip_channels[layer - 1]
                blocks[f"x_{depth}_{layer}"] = DecoderBlock(in_ch, skip_ch, out_ch, use_batchnorm, attention_type)
        last = len(self.in_channels) - 1
        blocks[f"x_0_{last}"] = DecoderBlock(self.in_channels[-1], 0, self.out_channels[-1], use_batchnorm,
                                             attention_type)
        self.blocks = nn.ModuleDict(blocks)
        self.depth = last

    def forward(self, *features):
        feats = list(features[1:])[::-1]
        dense = {}
        for layer in range(len(self.in_channels) - 1):
            for depth in range(self.depth - layer):
                if layer == 0:
                    dense[f"x_{depth}_{depth}"] = self.blocks[f"x_{depth}_{depth}"](feats[depth], feats[depth + 1])
                else:
                    li = depth + layer
                    cat = [dense[f"x_{k}_{li}"] for k in range(depth + 1, li + 1)] + [feats[li + 1]]
                    dtype = dense[f"x_{depth}_{li - 1}"].dtype
                    cat = torch.cat([c.to(dtype) for c in cat], dim=1)
                    dense[f"x_{depth}_{li}"] = self.blocks[f"x_{depth}_{li}"](dense[f"x_{depth}_{li - 1}"], cat)
        return self.blocks[f"x_0_{self.depth}"](dense[f"x_0_{self.depth - 1}"])


class UnetPlusPlus(SegmentationModel):
    def __init__(self, encoder_name="resnet34", encoder_depth=5, encoder_weights="imagenet", decoder_use_batchnorm=True,
                 decoder_channels=(256, 128, 64, 32, 16), decoder_attention_type=None, in_channels=3, classes=1):
        super().__init__()
        self.encoder = get_encoder(encoder_name, in_channels, encoder_depth, encoder_weights)
        self.decoder = UnetPlusPlusDecoder(self.encoder.out_channels, decoder_channels, encoder_depth,
                                           decoder_use_batchnorm, decoder_attention_type,
                                           center=encoder_name.startswith("vgg"))
        self.segmentation_head = SegmentationHead(decoder_channels[-1], classes, kernel_size=3)
        self.initialize()
