"""MA-Net decoder (SMP layout): position-wise attention block at the bottleneck and
multi-scale fusion attention (SE-style) blocks in the decoder.

Behavioural target: SMP ``MAnet`` (reference models/__init__.py:42-44).  The
PAB spatial map is a softmax over the whole flattened (HW x HW) map per
sample, as in SMP.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .base import Conv2dReLU, SegmentationHead, SegmentationModel
from .encoders import get_encoder
from .unet import _decoder_channels


class PAB(nn.Module):
    def __init__(self, in_channels, out_channels, pab_channels=64):
        super().__init__()
        self.pab_channels = pab_channels
        self.in_channels = in_channels
        self.top_conv = nn.Conv2d(in_channels, pab_channels, kernel_size=1)
        self.center_conv = nn.Conv2d(in_channels, pab_channels, kernel_size=1)
        self.bottom_conv = nn.Conv2d(in_channels, in_channels, kernel_size=3, padding=1)
        self.map_softmax = nn.Softmax(dim=1)
        self.out_conv = nn.Conv2d(in_channels, in_channels, kernel_size=3, padding=1)

    def forward(self, x):
        n, _, h, w = x.shape
        top = self.top_conv(x).flatten(2)                       # [N, P, HW]
        center = self.center_conv(x).flatten(2).transpose(1, 2)  # [N, HW, P]
        bottom = self.bottom_conv(x).flatten(2).transpose(1, 2)  # [N, HW, C]
        sp = torch.matmul(center, top)
        sp = torch.softmax(sp.reshape(n, -1).float(), dim=1).to(sp.dtype).reshape(n, h * w, h * w)
        sp = torch.matmul(sp, bottom).reshape(n, self.in_channels, h, w)
        return self.out_conv(x + sp.to(x.dtype))


def _se(channels, reduced):
    return nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(channels, reduced, 1), nn.ReLU(inplace=True),
                         nn.Conv2d(reduced, channels, 1), nn.Sigmoid())


class MFAB(nn.Module):
    def __init__(self, in_channels, skip_channels, out_channels, use_batchnorm=True, reduction=16):
        super().__init__()
        self.hl_conv = nn.Sequential(
            Conv2dReLU(in_channels, in_channels, 3, padding=1, use_batchnorm=use_batchnorm),
            Conv2dReLU(in_channels, skip_channels, 1, use_batchnorm=use_batchnorm))
        reduced = max(1, skip_channels // reduction)
        self.SE_ll = _se(skip_channels, reduced)
        self.SE_hl = _se(skip_channels, reduced)
        self.conv1 = Conv2dReLU(skip_channels + skip_channels, out_channels, 3, padding=1, use_batchnorm=use_batchnorm)
        self.conv2 = Conv2dReLU(out_channels, out_channels, 3, padding=1, use_batchnorm=use_batchnorm)

    def forward(self, x, skip=None):
        x = F.interpolate(self.hl_conv(x), scale_factor=2, mode="nearest")
        att = self.SE_hl(x)
        if skip is not None:
            att = att + self.SE_ll(skip)
            x = torch.cat([x * att, skip.to(x.dtype)], dim=1)
        return self.conv2(self.conv1(x))


class DecoderBlock(nn.Module):
    def __init__(self, in_channels, skip_channels, out_channels, use_batchnorm=True):
        super().__init__()
        self.conv1 = Conv2dReLU(in_channels + skip_channels, out_channels, 3, padding=1, use_batchnorm=use_batchnorm)
        self.conv2 = Conv2dReLU(out_channels, out_channels, 3, padding=1, use_batchnorm=use_batchnorm)

    def forward(self, x, skip=None):
        x = F.interpolate(x, scale_factor=2, mode="nearest")
        if skip is not None:
            x = torch.cat([x, skip.to(x.dtype)], dim=1)
        return self.conv2(self.conv1(x))


class MAnetDecoder(nn.Module):
    def __init__(self, encoder_channels, decoder_channels, n_blocks=5, reduction=16, use_batchnorm=True,
                 pab_channels=64):
        super().__init__()
        if n_blocks != len(decoder_channels):
            raise ValueError(f"Model depth is {n_blocks}, but you provide `decoder_channels` for "
                             f"{len(decoder_channels)} blocks.")
        enc, ins, skips, outs = _decoder_channels(encoder_channels, decoder_channels)
        self.center = PAB(enc[0], enc[0], pab_channels=pab_channels)
        self.blocks = nn.ModuleList([MFAB(i, s, o, use_batchnorm) if s > 0 else DecoderBlock(i, s, o, use_batchnorm)
                                     for i, s, o in zip(ins, skips, outs)])

    def forward(self, *features):
        feats = list(features[1:])[::-1]
        x = self.center(feats[0])
        skips = feats[1:]
        for i, blk in enumerate(self.blocks):
            x = blk(x, skips[i] if i < len(skips) else None)
        return x


class MAnet(SegmentationModel):
    def __init__(self, encoder_name="resnet34", encoder_depth=5, encoder_weights="imagenet", decoder_use_batchnorm=True,
                 decoder_channels=(256, 128, 64, 32, 16), decoder_pab_channels=64, in_channels=3, classes=1):
        super().__init__()
        self.encoder = get_encoder(encoder_name, in_channels, encoder_depth, encoder_weights)
        self.decoder = MAnetDecoder(self.encoder.out_channels, decoder_channels, encoder_depth,
                                    use_batchnorm=decoder_use_batchnorm, pab_channels=decoder_pab_channels)
        self.segmentation_head = SegmentationHead(decoder_channels[-1], classes, kernel_size=3)
        self.initialize()
