"""SQNet (ICLR-W 2017, "Speeding up semantic segmentation for autonomous driving").

Parity target: reference models/sqnet.py (SQNet :15-69 -- SqueezeNet-1.1
encoder, parallel dilated conv, deconv + bypass refinement decoder;
FireModule :72-86, ParallelDilatedConv :89-106, BypassRefinementModule :109-121).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .modules import ConvBNAct, DeConvBNAct

# (in, squeeze, expand1, expand3) of the Fire modules in each stage
_FIRE = (((64, 16, 64, 64), (128, 16, 64, 64)),
         ((128, 32, 128, 128), (256, 32, 128, 128)),
         ((256, 48, 192, 192), (384, 48, 192, 192), (384, 64, 256, 256), (512, 64, 256, 256)))


class SQNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="elu"):
        super().__init__()
        self.conv = ConvBNAct(n_channel, 64, 3, 2, act_type=act_type)
        for i, stage in enumerate(_FIRE, start=1):
            setattr(self, f"pool{i}", nn.MaxPool2d(3, 2, 1))
            setattr(self, f"fire{i}", nn.Sequential(*[FireModule(*cfg, act_type) for cfg in stage]))
        self.pdc = ParallelDilatedConv(512, 128, (1, 2, 4, 8), act_type)
        self.up1 = DeConvBNAct(128, 128, act_type=act_type)
        self.refine1 = BypassRefinementModule(256, 128, 128, act_type)
        self.up2 = DeConvBNAct(128, 128, act_type=act_type)
        self.refine2 = BypassRefinementModule(128, 128, 64, act_type=act_type)
        self.up3 = DeConvBNAct(64, 64, act_type=act_type)
        self.refine3 = BypassRefinementModule(64, 64, num_class, act_type=act_type)
        self.up4 = DeConvBNAct(num_class, num_class, act_type=act_type)

    def forward(self, x, is_training=False):
        x1 = self.conv(x)
        x2 = self.fire1(self.pool1(x1))
        x3 = self.fire2(self.pool2(x2))
        y = self.pdc(self.fire3(self.pool3(x3)))
        y = self.refine1(x3, self.up1(y))
        y = self.refine2(x2, self.up2(y))
        y = self.refine3(x1, self.up3(y))
        return self.up4(y)


class FireModule(nn.Module):
    def __init__(self, in_channels, sq_channels, ex1_channels, ex3_channels, act_type):
        super().__init__()
        self.conv_squeeze = ConvBNAct(in_channels, sq_channels, 1, act_type=act_type)
        self.conv_expand1 = ConvBNAct(sq_channels, ex1_channels, 1, act_type=act_type)
        self.conv_expand3 = ConvBNAct(sq_channels, ex3_channels, 3, act_type=act_type)

    def forward(self, x):
        s = self.conv_squeeze(x)
        return torch.cat([self.conv_expand1(s), self.conv_expand3(s)], dim=1)


class ParallelDilatedConv(nn.Module):
    def __init__(self, in_channels, out_channels, dilations, act_type):
        super().__init__()
        if len(dilations) != 4:
            raise AssertionError("Length of dilations should be 4.\n")
        for i, d in enumerate(dilations):
            setattr(self, f"conv{i}", ConvBNAct(in_channels, out_channels, 3, dilation=d, act_type=act_type))

    def forward(self, x):
        return self.conv0(x) + self.conv1(x) + self.conv2(x) + self.conv3(x)


class BypassRefinementModule(nn.Module):
    def __init__(self, low_channels, high_channels, out_channels, act_type):
        super().__init__()
        self.conv_low = ConvBNAct(low_channels, low_channels, 3, act_type=act_type)
        self.conv_cat = ConvBNAct(low_channels + high_channels, out_channels, 3, act_type=act_type)

    def forward(self, x_low, x_high):
        return self.conv_cat(torch.cat([self.conv_low(x_low), x_high], dim=1))
