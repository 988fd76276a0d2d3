"""CGNet (arXiv:1811.08201) -- context guided network.

Parity target: reference models/cgnet.py (CGNet :15-47 with image injection at
1/4 and 1/8, InitBlock :50-61, build_blocks :64-69, CGBlock :72-113 -- local
(depth-wise) + surrounding (dilated depth-wise) features, joint BN+act, global
SE-style reweighting, GRL/LRL residual).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .modules import Activation, ConvBNAct, conv1x1


class CGNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, M=3, N=15, act_type="prelu"):
        super().__init__()
        self.stage1 = InitBlock(n_channel, 32, act_type=act_type)
        self.stage2_down = CGBlock(64, 64, 2, 2, act_type=act_type)
        self.stage2 = build_blocks(CGBlock, 64 + 3, 64, 2, M - 1, act_type)
        self.stage3_down = CGBlock(128, 128, 2, 4, act_type=act_type)
        self.stage3 = build_blocks(CGBlock, 128 + 3, 128, 4, N - 1, act_type)
        self.seg_head = conv1x1(128 * 2, num_class)

    def forward(self, x, is_training=False):
        h, w = x.shape[2:]
        x_d4 = ops.interpolate(x, (h // 4, w // 4), True)
        x_d8 = ops.interpolate(x, (h // 8, w // 8), True)
        y, y0 = self.stage1(x)
        x2 = self.stage2_down(torch.cat([y, y0], dim=1))
        y = self.stage2(torch.cat([x2, x_d4], dim=1))
        x3 = self.stage3_down(torch.cat([y, x2], dim=1))
        y = self.stage3(torch.cat([x3, x_d8], dim=1))
        return ops.final_upsample(self.seg_head(torch.cat([y, x3], dim=1)), (h, w), True)


class InitBlock(nn.Module):
    def __init__(self, in_channels, out_channels, act_type):
        super().__init__()
        self.conv0 = ConvBNAct(in_channels, out_channels, stride=2, act_type=act_type)
        self.conv1 = ConvBNAct(out_channels, out_channels, act_type=act_type)
        self.conv2 = ConvBNAct(out_channels, out_channels, act_type=act_type)

    def forward(self, x):
        x0 = self.conv0(x)
        return self.conv2(self.conv1(x0)), x0


def build_blocks(block, in_channels, out_channels, dilation, num_block, act_type):
    layers = []
    for _ in range(num_block):
        layers.append(block(in_channels, out_channels, 1, dilation, act_type=act_type))
        in_channels = out_channels
    return nn.Sequential(*layers)


class CGBlock(nn.Module):
    def __init__(self, in_channels, out_channels, stride, dilation, res_type="GRL", act_type="prelu"):
        super().__init__()
        if res_type not in ("GRL", "LRL"):
            raise ValueError("Residual learning only support GRL and LRL type.\n")
        self.res_type = res_type
        self.use_skip = stride == 1 and in_channels == out_channels
        h = out_channels // 2
        self.conv = conv1x1(in_channels, h)
        self.loc = nn.Conv2d(h, h, 3, stride, padding=1, groups=h, bias=False)
        self.sur = nn.Conv2d(h, h, 3, stride, padding=dilation, dilation=dilation, groups=h, bias=False)
        self.joi = nn.Sequential(nn.BatchNorm2d(out_channels), Activation(act_type))
        self.glo = nn.Sequential(nn.Linear(out_channels, out_channels // 8),
                                 nn.Linear(out_channels // 8, out_channels))

    def forward(self, x):
        p = self.conv(x)
        # BN(+PReLU) of the joint feature loc || sur, the concat never materialised (ops.cat_bn_act)
        y = ops.cat_bn_act([self.loc(p), self.sur(p)], self.joi[0], self.joi[1], act_module=self.joi[1])
        if self.use_skip and self.res_type == "LRL":
            y = y + x
        y = ops.gate(y, self.glo(y.mean(dim=(2, 3)))[:, :, None, None], sigmoid=True)
        if self.use_skip and self.res_type == "GRL":
            y = y + x
        return y
