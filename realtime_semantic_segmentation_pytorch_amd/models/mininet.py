"""MiniNet (ICRA 2019, V-SLAM keyframe selection ConvNet).

Parity target: reference models/mininet.py (MiniNet :15-79 -- four
depth-wise separable downsamplers, dilated ConvModule branch, a deeper 1/32
branch, deconv decoder with skip concatenation; ConvModule :82-113 --
factorized depth-wise convs with inner/outer residuals and dropout).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .modules import Activation, DeConvBNAct, DSConvBNAct, conv1x1


class MiniNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="selu"):
        super().__init__()
        chans = (n_channel, 12, 24, 48, 96)
        for i in range(1, 5):
            setattr(self, f"down{i}", DSConvBNAct(chans[i - 1], chans[i], 3, 2, act_type=act_type))
        self.branch1 = nn.Sequential(*[ConvModule(96, d, act_type) for d in (1, 2, 4, 8)])
        self.branch2_down = DSConvBNAct(96, 192, 3, 2, act_type=act_type)
        self.branch2 = nn.Sequential(ConvModule(192, 1, act_type), DSConvBNAct(192, 386, 3, 2, act_type=act_type),
                                     ConvModule(386, 1, act_type), ConvModule(386, 1, act_type),
                                     DeConvBNAct(386, 192, act_type=act_type), ConvModule(192, 1, act_type))
        self.branch2_up = DeConvBNAct(192 * 2, 96, act_type=act_type)
        self.up4 = nn.Sequential(DeConvBNAct(96 * 3, 96, act_type=act_type), ConvModule(96, 1, act_type),
                                 conv1x1(96, 48))
        self.up3 = DeConvBNAct(48 * 2, 24, act_type=act_type)
        self.up2 = DeConvBNAct(24 * 2, 12, act_type=act_type)
        self.up1 = DeConvBNAct(12 * 2, num_class, act_type=act_type)

    def forward(self, x, is_training=False):
        d1 = self.down1(x)
        d2 = self.down2(d1)
        d3 = self.down3(d2)
        d4 = self.down4(d3)
        b1 = self.branch1(d4)
        d5 = self.branch2_down(d4)
        b2 = self.branch2_up(torch.cat([self.branch2(d5), d5], dim=1))
        y = self.up4(torch.cat([b1, b2, d4], dim=1))
        y = self.up3(torch.cat([y, d3], dim=1))
        y = self.up2(torch.cat([y, d2], dim=1))
        return self.up1(torch.cat([y, d1], dim=1))


def _dw(channels, k, dilation):
    pad = tuple((kk - 1) // 2 * dilation for kk in k)
    return nn.Conv2d(channels, channels, k, padding=pad, dilation=dilation, groups=channels, bias=False)


class ConvModule(nn.Module):
    def __init__(self, channels, dilation, act_type):
        super().__init__()
        c, d = channels, dilation
        self.conv1 = nn.Sequential(_dw(c, (1, 3), d), Activation(act_type), _dw(c, (3, 1), d), Activation(act_type))
        self.conv2 = nn.Sequential(_dw(c, (3, 1), d), Activation(act_type), _dw(c, (1, 3), d))
        self.dropout = nn.Dropout(p=0.25)
        self.act = Activation(act_type)

    def forward(self, x):
        h = self.conv1(x)
        return self.act(self.dropout(self.conv2(h) + h) + x)
