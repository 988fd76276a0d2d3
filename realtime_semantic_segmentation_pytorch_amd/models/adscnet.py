"""ADSCNet (Applied Intelligence 2020) -- asymmetric depth-wise separable convs + DDCC.

Parity target: reference models/adscnet.py (ADSCNet :15-53, ADSCModule
:56-80 -- residual for stride 1, conv || avg-pool concat for stride 2; DDCC
:83-125 densely-connected dilated (avg-pool + ADSC) blocks).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .modules import ConvBNAct, DeConvBNAct, DWConvBNAct, conv1x1


class ADSCNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="relu6"):
        super().__init__()
        self.conv0 = ConvBNAct(n_channel, 32, 3, 2, act_type=act_type, inplace=True)
        self.conv1 = ADSCModule(32, 1, act_type=act_type)
        self.conv2_4 = nn.Sequential(ADSCModule(32, 1, act_type=act_type), ADSCModule(32, 2, act_type=act_type),
                                     ADSCModule(64, 1, act_type=act_type))
        self.conv5 = ADSCModule(64, 2, act_type=act_type)
        self.ddcc = DDCC(128, (3, 5, 9, 13), act_type)
        self.up1 = nn.Sequential(DeConvBNAct(128, 64), ADSCModule(64, 1, act_type=act_type))
        self.up2 = nn.Sequential(ADSCModule(64, 1, act_type=act_type), DeConvBNAct(64, 32))
        self.up3 = nn.Sequential(ADSCModule(32, 1, act_type=act_type), DeConvBNAct(32, num_class))

    def forward(self, x, is_training=False):
        x1 = self.conv1(self.conv0(x))
        x4 = self.conv2_4(x1)
        y = self.up1(self.ddcc(self.conv5(x4))) + x4
        y = self.up2(y) + x1
        return self.up3(y)


class ADSCModule(nn.Module):
    def __init__(self, channels, stride, dilation=1, act_type="relu"):
        super().__init__()
        if stride not in (1, 2):
            raise AssertionError("Unsupported stride type.\n")
        self.use_skip = stride == 1
        self.conv = nn.Sequential(
            DWConvBNAct(channels, channels, (3, 1), stride, dilation, act_type, inplace=True),
            conv1x1(channels, channels),
            DWConvBNAct(channels, channels, (1, 3), 1, dilation, act_type, inplace=True),
            conv1x1(channels, channels))
        if not self.use_skip:
            self.pool = nn.AvgPool2d(3, 2, 1)

    def forward(self, x):
        y = self.conv(x)
        return x + y if self.use_skip else torch.cat([y, self.pool(x)], dim=1)


class DDCC(nn.Module):
    """Dense dilated cascade: block i sees concat(x, outputs of blocks < i)."""

    def __init__(self, channels, dilations, act_type):
        super().__init__()
        if len(dilations) != 4:
            raise AssertionError("Length of dilations should be 4.\n")
        for i, d in enumerate(dilations, start=1):
            mods = [conv1x1(i * channels, channels)] if i > 1 else []
            mods += [nn.AvgPool2d(d, 1, d // 2), ADSCModule(channels, 1, d, act_type)]
            setattr(self, f"block{i}", nn.Sequential(*mods))
        self.conv_last = conv1x1(5 * channels, channels)

    def forward(self, x):
        feats = [x]
        for i in range(1, 5):
            blk = getattr(self, f"block{i}")
            feats.append(blk(feats[0] if i == 1 else torch.cat(feats, dim=1)))
        return self.conv_last(torch.cat(feats, dim=1))
