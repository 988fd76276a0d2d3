"""EDANet (arXiv:1809.06323) -- efficient dense modules of asymmetric convolution.

Parity target: reference models/edanet.py (EDANet :15-35, DownsamplingBlock
:38-50 (conv || max-pool, then BN+act), EDABlock :53-66, EDAModule :69-85 --
dense concatenation of k new channels per module).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .modules import Activation, ConvBNAct, conv1x1, conv3x3


class EDANet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, k=40, num_b1=5, num_b2=8, act_type="relu"):
        super().__init__()
        self.stage1 = DownsamplingBlock(n_channel, 15, act_type)
        self.stage2_d = DownsamplingBlock(15, 60, act_type)
        self.stage2 = EDABlock(60, k, num_b1, (1, 1, 1, 2, 2), act_type)
        self.stage3_d = ConvBNAct(60 + k * num_b1, 130, 3, 2, act_type=act_type)
        self.stage3 = EDABlock(130, k, num_b2, (2, 2, 4, 4, 8, 8, 16, 16), act_type)
        self.project = conv1x1(130 + k * num_b2, num_class)

    def forward(self, x, is_training=False):
        y = self.stage3(self.stage3_d(self.stage2(self.stage2_d(self.stage1(x)))))
        return ops.final_upsample(self.project(y), x.shape[2:], True)


class DownsamplingBlock(nn.Module):
    def __init__(self, in_channels, out_channels, act_type):
        super().__init__()
        self.conv = conv3x3(in_channels, out_channels - in_channels, 2)
        self.pool = nn.MaxPool2d(2, 2)
        self.bn_act = nn.Sequential(nn.BatchNorm2d(out_channels), Activation(act_type))

    def forward(self, x):
        c = self.conv(x)  # (autocast: the pooled fp32 input joins in the conv's dtype, see enet.InitialBlock)
        # BN + act of conv || pool straight into the concat layout (ops.cat_bn_act)
        return ops.cat_bn_act([c, self.pool(x).to(c.dtype)], self.bn_act[0], self.bn_act[1],
                              act_module=self.bn_act[1])


class EDABlock(nn.Module):
    def __init__(self, in_channels, k, num_block, dilations, act_type):
        super().__init__()
        if len(dilations) != num_block:
            raise AssertionError("number of dilation rate should be equal to number of block")
        mods = []
        for i, d in enumerate(dilations):
            mods.append(EDAModule(in_channels + i * k, k, d, act_type))
        self.layers = nn.Sequential(*mods)

    def forward(self, x):
        return self.layers(x)


class EDAModule(nn.Module):
    """1x1 -> (3,1),(1,3) -> dilated (3,1),(1,3); output concatenated in front of the input."""

    def __init__(self, in_channels, k, dilation=1, act_type="relu"):
        super().__init__()
        d = dilation
        self.conv = nn.Sequential(
            ConvBNAct(in_channels, k, 1),
            nn.Conv2d(k, k, (3, 1), padding=(1, 0), bias=False),
            ConvBNAct(k, k, (1, 3), act_type=act_type),
            nn.Conv2d(k, k, (3, 1), dilation=d, padding=(d, 0), bias=False),
            ConvBNAct(k, k, (1, 3), dilation=d, act_type=act_type))

    def forward(self, x):
        y = self.conv(x)
        return torch.cat([y, x.to(y.dtype)], dim=1)
