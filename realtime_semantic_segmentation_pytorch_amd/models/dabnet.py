"""DABNet (arXiv:1907.11357) -- depth-wise asymmetric bottleneck network.

Parity target: reference models/dabnet.py (DABNet :16-61 with average-pooled
image injection at 1/2, 1/4, 1/8; build_blocks :64-68; DABModule :71-98 --
3x3 reduce, plain and dilated depth-wise (3,1)/(1,3) branches, 1x1 expand,
residual).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .enet import InitialBlock
from .modules import ConvBNAct, DWConvBNAct, conv1x1


def build_blocks(block, channels, num_block, dilation, act_type):
    return nn.Sequential(*[block(channels, dilation, act_type=act_type) for _ in range(num_block)])


class DABNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="prelu"):
        super().__init__()
        self.layer1 = ConvBNAct(n_channel, 32, 3, 2, act_type=act_type)
        self.layer2 = ConvBNAct(32, 32, 3, 1, act_type=act_type)
        self.layer3 = ConvBNAct(32, 32, 3, 1, act_type=act_type)
        self.layer4 = InitialBlock(32 + n_channel, 64, act_type=act_type)
        self.layer5_7 = build_blocks(DABModule, 64, 3, dilation=2, act_type=act_type)
        self.layer8 = ConvBNAct(64 * 2 + n_channel, 128, 3, 2, act_type=act_type)
        self.layer9_10 = build_blocks(DABModule, 128, 2, dilation=4, act_type=act_type)
        self.layer11_12 = build_blocks(DABModule, 128, 2, dilation=8, act_type=act_type)
        self.layer13_14 = build_blocks(DABModule, 128, 2, dilation=16, act_type=act_type)
        self.layer15 = conv1x1(128 * 2 + n_channel, num_class)

    def forward(self, x, is_training=False):
        pyr = [x]
        for _ in range(3):  # image pyramid for input injection
            pyr.append(F.avg_pool2d(pyr[-1], 3, 2, 1))
        y = torch.cat([self.layer3(self.layer2(self.layer1(x))), pyr[1]], dim=1)
        b1 = self.layer4(y)
        y = torch.cat([self.layer5_7(b1), b1, pyr[2]], dim=1)
        b2 = self.layer8(y)
        y = self.layer13_14(self.layer11_12(self.layer9_10(b2)))
        y = self.layer15(torch.cat([y, b2, pyr[3]], dim=1))
        return ops.final_upsample(y, x.shape[2:], True)


class DABModule(nn.Module):
    def __init__(self, channels, dilation, act_type):
        super().__init__()
        if channels % 2:
            raise AssertionError("Input channel of DABModule should be multiple of 2.\n")
        h = channels // 2
        self.init_conv = ConvBNAct(channels, h, 3, act_type=act_type)
        self.left_branch = nn.Sequential(DWConvBNAct(h, h, (3, 1), act_type=act_type),
                                         DWConvBNAct(h, h, (1, 3), act_type=act_type))
        self.right_branch = nn.Sequential(DWConvBNAct(h, h, (3, 1), dilation=dilation, act_type=act_type),
                                          DWConvBNAct(h, h, (1, 3), dilation=dilation, act_type=act_type))
        self.last_conv = ConvBNAct(h, channels, 1, act_type=act_type)

    def forward(self, x):
        y = self.init_conv(x)
        return self.last_conv(self.left_branch(y) + self.right_branch(y)) + x
