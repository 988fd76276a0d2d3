"""ERFNet (IEEE T-ITS 2018, "Efficient residual factorized ConvNet").

Parity target: reference models/erfnet.py (ERFNet :15-46 with ENet-style
downsampler blocks, build_blocks :49-59, NonBt1DBlock :62-82 -- factorized
(3,1)/(1,3) convs, the second pair dilated, residual before BN+act).
"""
from __future__ import annotations

import torch.nn as nn

from .. import ops
from .enet import InitialBlock as DownsamplerBlock
from .modules import Activation, ConvBNAct, DeConvBNAct


def build_blocks(block, channels, num_block, dilations=(), act_type="relu"):
    dilations = list(dilations) or [1] * num_block
    if len(dilations) != num_block:
        raise ValueError("Number of dilation should be equal to number of blocks")
    return nn.Sequential(*[block(channels, dilation=d, act_type=act_type) for d in dilations])


class ERFNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="relu"):
        super().__init__()
        self.layer1 = DownsamplerBlock(n_channel, 16, act_type=act_type)
        self.layer2 = DownsamplerBlock(16, 64, act_type=act_type)
        self.layer3_7 = build_blocks(NonBt1DBlock, 64, 5, act_type=act_type)
        self.layer8 = DownsamplerBlock(64, 128, act_type=act_type)
        self.layer9_16 = build_blocks(NonBt1DBlock, 128, 8, dilations=(2, 4, 8, 16) * 2, act_type=act_type)
        self.layer17 = DeConvBNAct(128, 64, act_type=act_type)
        self.layer18_19 = build_blocks(NonBt1DBlock, 64, 2, act_type=act_type)
        self.layer20 = DeConvBNAct(64, 16, act_type=act_type)
        self.layer21_22 = build_blocks(NonBt1DBlock, 16, 2, act_type=act_type)
        self.layer23 = DeConvBNAct(16, num_class, act_type=act_type)

    def forward(self, x, is_training=False):
        for name in ("layer1", "layer2", "layer3_7", "layer8", "layer9_16", "layer17", "layer18_19",
                     "layer20", "layer21_22", "layer23"):
            x = getattr(self, name)(x)
        return x


class NonBt1DBlock(nn.Module):
    def __init__(self, channels, dilation=1, act_type="relu"):
        super().__init__()
        d = dilation
        self.conv = nn.Sequential(
            ConvBNAct(channels, channels, (3, 1), inplace=True),
            ConvBNAct(channels, channels, (1, 3), inplace=True),
            ConvBNAct(channels, channels, (3, 1), dilation=d, inplace=True),
            nn.Conv2d(channels, channels, (1, 3), dilation=d, padding=(0, d), bias=False))
        self.bn_act = nn.Sequential(nn.BatchNorm2d(channels), Activation(act_type, inplace=True))

    def forward(self, x):
        # act(BN(conv(x) + x)): the sum feeds the BN, so BN+act fuse on the sum
        bn, act = self.bn_act[0], self.bn_act[1]
        return ops.bn_act(self.conv(x) + x, bn, act, act_module=act)
