"""FDDWNet (arXiv:1911.00632) -- factorized dilated depth-wise separable convs.

Parity target: reference models/fddwnet.py (FDDWNet :16-47, build_blocks
:50-61, EERMUnit :64-85 -- two factorized depth-wise pairs each followed by a
1x1 ConvBNAct, residual + act).
"""
from __future__ import annotations

import torch.nn as nn

from .enet import InitialBlock as DownsamplingUnit
from .modules import Activation, ConvBNAct, DeConvBNAct, DWConvBNAct


class FDDWNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, ks=3, act_type="relu"):
        super().__init__()
        self.layer1 = DownsamplingUnit(n_channel, 16, act_type)
        self.layer2 = DownsamplingUnit(16, 64, act_type)
        self.layer3_7 = build_blocks(EERMUnit, 64, 5, ks, (1,) * 5, act_type)
        self.layer8 = DownsamplingUnit(64, 128, act_type)
        self.layer9_16 = build_blocks(EERMUnit, 128, 8, ks, (1, 2, 5, 9, 1, 2, 5, 9), act_type)
        self.layer17_24 = build_blocks(EERMUnit, 128, 8, ks, (2, 5, 9, 17, 2, 5, 9, 17), act_type)
        self.layer25 = DeConvBNAct(128, 64, act_type=act_type)
        self.layer26_27 = build_blocks(EERMUnit, 64, 2, ks, (1, 1), act_type)
        self.layer28 = DeConvBNAct(64, 16, act_type=act_type)
        self.layer29_30 = build_blocks(EERMUnit, 16, 2, ks, (1, 1), act_type)
        self.layer31 = DeConvBNAct(16, num_class, act_type=act_type)

    def forward(self, x, is_training=False):
        skip = self.layer3_7(self.layer2(self.layer1(x)))
        y = self.layer17_24(self.layer9_16(self.layer8(skip)))
        y = self.layer26_27(self.layer25(y)) + skip
        return self.layer31(self.layer29_30(self.layer28(y)))


def build_blocks(block, channels, num_block, kernel_size, dilations=(), act_type="relu"):
    dilations = list(dilations) or [1] * num_block
    if len(dilations) != num_block:
        raise ValueError("Number of dilation should be equal to number of blocks")
    return nn.Sequential(*[block(channels, kernel_size, d, act_type) for d in dilations])


class EERMUnit(nn.Module):
    def __init__(self, channels, ks, dt, act_type):
        super().__init__()
        c = channels
        self.conv = nn.Sequential(
            DWConvBNAct(c, c, (ks, 1), act_type="none"),
            DWConvBNAct(c, c, (1, ks), act_type="none"),
            ConvBNAct(c, c, 1, act_type=act_type, inplace=True),
            DWConvBNAct(c, c, (ks, 1), dilation=dt, act_type="none"),
            DWConvBNAct(c, c, (1, ks), dilation=dt, act_type="none"),
            ConvBNAct(c, c, 1, act_type="none"))
        self.act = Activation(act_type)

    def forward(self, x):
        h = x
        for m in list(self.conv)[:5]:
            h = m(h)
        return self.conv[5](h, residual=x, act=self.act)
