"""FSSNet (IEEE T-II 2018, "Fast semantic segmentation for scene perception").

Parity target: reference models/fssnet.py (FSSNet :16-46, build_blocks
:49-59, FactorizedBlock :62-82, DilatedBlock :85-103, DownsamplingBlock
:106-128, UpsamplingBlock :131-157).  Residual adds are fused into the last
BN of each block; the decoder's x2 resize fuses the deconv-branch add.
"""
from __future__ import annotations

import torch.nn as nn

from .. import ops
from .enet import InitialBlock as InitBlock
from .modules import Activation, ConvBNAct, DeConvBNAct


class FSSNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="prelu"):
        super().__init__()
        self.init_block = InitBlock(n_channel, 16, act_type)
        self.down1 = DownsamplingBlock(16, 64, act_type)
        self.factorized = build_blocks(FactorizedBlock, 64, 4, act_type=act_type)
        self.down2 = DownsamplingBlock(64, 128, act_type)
        self.dilated = build_blocks(DilatedBlock, 128, 6, (2, 5, 9, 2, 5, 9), act_type)
        self.up2 = UpsamplingBlock(128, 64, act_type)
        self.bottleneck2 = build_blocks(DilatedBlock, 64, 2, act_type=act_type)
        self.up1 = UpsamplingBlock(64, 16, act_type)
        self.bottleneck1 = build_blocks(DilatedBlock, 16, 2, act_type=act_type)
        self.full_conv = DeConvBNAct(16, num_class, act_type=act_type)

    def forward(self, x, is_training=False):
        d1 = self.down1(self.init_block(x))  # 1/4
        d2 = self.down2(self.factorized(d1))  # 1/8
        y = self.bottleneck2(self.up2(self.dilated(d2), d2))
        y = self.bottleneck1(self.up1(y, d1))
        return self.full_conv(y)


def build_blocks(block, channels, num_block, dilations=(), act_type="relu"):
    dilations = list(dilations) or [1] * num_block
    if len(dilations) != num_block:
        raise ValueError("Number of dilation should be equal to number of blocks")
    return nn.Sequential(*[block(channels, d, act_type) for d in dilations])


class _ResidualTail(nn.Module):
    """act(conv(x) + x) with BN(+residual)+act fused in the last ConvBNAct."""

    def forward(self, x):
        h = x
        for m in list(self.conv)[:-1]:
            h = m(h)
        return self.conv[-1](h, residual=x, act=self.act)


class FactorizedBlock(_ResidualTail):
    def __init__(self, channels, dilation=1, act_type="relu"):
        super().__init__()
        h = channels // 4
        self.conv = nn.Sequential(ConvBNAct(channels, h, 1, act_type=act_type),
                                  ConvBNAct(h, h, (1, 3), act_type="none"),
                                  ConvBNAct(h, h, (3, 1), act_type=act_type),
                                  ConvBNAct(h, channels, 1, act_type="none"))
        self.act = Activation(act_type)


class DilatedBlock(_ResidualTail):
    def __init__(self, channels, dilation, act_type):
        super().__init__()
        h = channels // 4
        self.conv = nn.Sequential(ConvBNAct(channels, h, 1, act_type=act_type),
                                  ConvBNAct(h, h, 3, dilation=dilation, act_type=act_type),
                                  ConvBNAct(h, channels, 1, act_type="none"))
        self.act = Activation(act_type)


class DownsamplingBlock(nn.Module):
    def __init__(self, in_channels, out_channels, act_type):
        super().__init__()
        h = out_channels // 4
        self.conv = nn.Sequential(ConvBNAct(in_channels, h, 2, 2, act_type=act_type),
                                  ConvBNAct(h, h, 3, act_type=act_type),
                                  ConvBNAct(h, out_channels, 1, act_type="none"))
        self.pool = nn.Sequential(nn.MaxPool2d(3, 2, 1), ConvBNAct(in_channels, out_channels, 1, act_type="none"))
        self.act = Activation(act_type)

    def forward(self, x):
        p = self.pool(x)
        return self.conv[2](self.conv[1](self.conv[0](x)), residual=p, act=self.act)


class UpsamplingBlock(nn.Module):
    def __init__(self, in_channels, out_channels, act_type):
        super().__init__()
        h = in_channels // 4
        self.deconv = nn.Sequential(ConvBNAct(in_channels, h, 1, act_type=act_type),
                                    DeConvBNAct(h, h, act_type=act_type),
                                    ConvBNAct(h, out_channels, 1, act_type="none"))
        self.conv = ConvBNAct(in_channels, out_channels, 1, act_type="none")
        self.act = Activation(act_type)

    def forward(self, x, pool_feat):
        d = self.deconv(x)
        y = self.conv(x + pool_feat)
        return self.act(ops.interpolate(y, d.shape[2:], True, skip=d))
