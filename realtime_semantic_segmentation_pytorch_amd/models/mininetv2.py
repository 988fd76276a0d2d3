"""MiniNet-v2 (ICRA 2020, "MiniNet: an efficient semantic segmentation ConvNet").

Parity target: reference models/mininetv2.py (MiniNetv2 :16-48 -- a
refinement branch of two downsamplers added to the decoder; build_blocks
:51-61; MultiDilationDSConv :64-82 -- plain + dilated depth-wise sum then 1x1).
"""
from __future__ import annotations

import torch.nn as nn

from .. import ops
from .enet import InitialBlock as DownsamplingUnit
from .modules import DeConvBNAct, DWConvBNAct, PWConvBNAct

FEATURE_DILATIONS = (1, 2, 1, 4, 1, 8, 1, 16, 1, 1, 1, 2, 1, 4, 1, 8)


class MiniNetv2(nn.Module):
    def __init__(self, num_class=1, n_channel=3, feat_dt=FEATURE_DILATIONS, act_type="relu"):
        super().__init__()
        self.d1_2 = nn.Sequential(DownsamplingUnit(n_channel, 16, act_type), DownsamplingUnit(16, 64, act_type))
        self.ref = nn.Sequential(DownsamplingUnit(n_channel, 16, act_type), DownsamplingUnit(16, 64, act_type))
        self.m1_10 = build_blocks(MultiDilationDSConv, 64, 10, act_type=act_type)
        self.d3 = DownsamplingUnit(64, 128, act_type)
        self.feature_extractor = build_blocks(MultiDilationDSConv, 128, len(feat_dt), feat_dt, act_type)
        self.up1 = DeConvBNAct(128, 64, act_type=act_type)
        self.m26_29 = build_blocks(MultiDilationDSConv, 64, 4, act_type=act_type)
        self.output = DeConvBNAct(64, num_class, act_type=act_type)

    def forward(self, x, is_training=False):
        r = self.ref(x)
        y = self.feature_extractor(self.d3(self.m1_10(self.d1_2(x))))
        y = self.output(self.m26_29(self.up1(y) + r))
        return ops.final_upsample(y, x.shape[2:], True)


def build_blocks(block, channels, num_block, dilations=(), act_type="relu"):
    dilations = list(dilations) or [1] * num_block
    if len(dilations) != num_block:
        raise ValueError("Number of dilation should be equal to number of blocks")
    return nn.Sequential(*[block(channels, channels, 3, 1, d, act_type) for d in dilations])


class MultiDilationDSConv(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, dilation=1, act_type="relu"):
        super().__init__()
        self.dilated = dilation > 1
        self.dw_conv = DWConvBNAct(in_channels, in_channels, kernel_size, stride, 1, act_type)
        self.pw_conv = PWConvBNAct(in_channels, out_channels, act_type, inplace=True)
        if self.dilated:
            self.ddw_conv = DWConvBNAct(in_channels, in_channels, kernel_size, stride, dilation, act_type,
                                        inplace=True)

    def forward(self, x):
        h = self.dw_conv(x)
        if self.dilated:
            h = h + self.ddw_conv(x)
        return self.pw_conv(h)
