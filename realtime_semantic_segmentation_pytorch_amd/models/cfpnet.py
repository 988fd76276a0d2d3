"""CFPNet (arXiv:2103.12212) -- channel-wise feature pyramid.

Parity target: reference models/cfpnet.py (CFPNet :17-53 with bilinear image
pyramid injection, build_blocks :56-66, CFPModule :69-106 -- K feature-pyramid
channels with hierarchical sums, FeaturePyramidChannel :109-138).
"""
from __future__ import annotations

from math import ceil

import torch
import torch.nn as nn

from .. import ops
from .enet import InitialBlock as DownsamplingBlock
from .modules import ConvBNAct


class CFPNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, n=2, m=6, dilations=(2, 2, 4, 4, 8, 8, 16, 16),
                 act_type="prelu"):
        super().__init__()
        if len(dilations) != n + m:
            raise AssertionError(f"Length of dilations should be equal to {n + m}.\n")
        self.conv_init = nn.Sequential(ConvBNAct(n_channel, 32, stride=2, act_type=act_type),
                                       ConvBNAct(32, 32, act_type=act_type),
                                       ConvBNAct(32, 32, act_type=act_type))
        self.downsample1 = DownsamplingBlock(32 + 3, 64, act_type)
        self.cfp1 = build_blocks(CFPModule, 64, n, dilations[:n], act_type)
        self.downsample2 = DownsamplingBlock(64 + 3, 128, act_type)
        self.cfp2 = build_blocks(CFPModule, 128, m, dilations[n:], act_type)
        self.seg_head = ConvBNAct(128 + 3, num_class, 1, act_type=act_type)

    def forward(self, x, is_training=False):
        h, w = x.shape[2:]
        # align_corners=True ignores the scale factor in the coordinate map, so a size suffices
        pyr = [ops.interpolate(x, (h // f, w // f), True) for f in (2, 4, 8)]
        y = self.downsample1(torch.cat([self.conv_init(x), pyr[0]], dim=1))
        y = self.downsample2(torch.cat([self.cfp1(y), pyr[1]], dim=1))
        y = self.seg_head(torch.cat([self.cfp2(y), pyr[2]], dim=1))
        return ops.final_upsample(y, (h, w), True)


def build_blocks(block, channels, num_block, dilations=(), act_type="relu"):
    dilations = list(dilations) or [1] * num_block
    if len(dilations) != num_block:
        raise ValueError("Number of dilation should be equal to number of blocks")
    return nn.Sequential(*[block(channels, d, act_type=act_type) for d in dilations])


class CFPModule(nn.Module):
    def __init__(self, channels, rk, K=4, rk_ratio=None, act_type="prelu"):
        super().__init__()
        rk_ratio = rk_ratio or (1 / rk, 1 / 4, 1 / 2, 1)
        if len(rk_ratio) != K:
            raise AssertionError(f"Length of rk_ratio should be {K}.\n")
        self.K = K
        ckn = channels // K
        self.conv_init = ConvBNAct(channels, ckn, 1, act_type=act_type)
        self.layers = nn.ModuleList([FeaturePyramidChannel(ckn, ceil(rk * r), act_type=act_type)
                                     for r in rk_ratio])
        self.conv_last = ConvBNAct(channels, channels, 1, act_type=act_type)

    def forward(self, x):
        p = self.conv_init(x)
        feats, run = [], None
        for layer in self.layers:  # hierarchical feature fusion: running sum over branches
            run = layer(p) if run is None else layer(p) + run
            feats.append(run)
        return self.conv_last(torch.cat(feats, dim=1)) + x


class FeaturePyramidChannel(nn.Module):
    def __init__(self, channels, dilation, act_type, channel_split=(1, 1, 2)):
        super().__init__()
        parts = sum(channel_split)
        if channels % parts:
            raise AssertionError(f"Channel of FPC should be multiple of {parts}.\n")
        widths = [channels // parts * s for s in channel_split]
        cin = channels
        for i, c in enumerate(widths, start=1):
            setattr(self, f"block{i}", nn.Sequential(
                ConvBNAct(cin, c, (3, 1), dilation=dilation, act_type=act_type),
                ConvBNAct(c, c, (1, 3), dilation=dilation, act_type=act_type)))
            cin = c

    def forward(self, x):
        x1 = self.block1(x)
        x2 = self.block2(x1)
        return torch.cat([x1, x2, self.block3(x2)], dim=1)
