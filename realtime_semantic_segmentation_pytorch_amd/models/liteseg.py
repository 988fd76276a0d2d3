"""LiteSeg (arXiv:1912.06683).

Parity target: reference models/liteseg.py (LiteSeg :16-44 with MobileNetV2 /
ResNet backbone, DASPPModule :47-73 -- dilated (3, 6, 9) + global-pool ASPP
with the input re-concatenated, SegHead :76-82).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .modules import ConvBNAct, conv1x1
from .swiftnet import make_backbone


class LiteSeg(nn.Module):
    def __init__(self, num_class=1, n_channel=3, backbone_type="mobilenet_v2", act_type="relu",
                 pretrained=False):
        super().__init__()
        self.backbone, ch = make_backbone(backbone_type, pretrained)
        self.daspp = DASPPModule(ch[3], 512, act_type)
        self.seg_head = SegHead(512 + ch[1], num_class, act_type)

    def forward(self, x, is_training=False):
        _, x8, _, x32 = self.backbone(x)
        y = ops.interpolate(self.daspp(x32), x8.shape[2:], True)
        y = self.seg_head(torch.cat([y, x8], dim=1))
        return ops.final_upsample(y, x.shape[2:], True)


class DASPPModule(nn.Module):
    DILATIONS = (3, 6, 9)

    def __init__(self, in_channels, out_channels, act_type):
        super().__init__()
        hid = in_channels // 5
        self.stage1 = ConvBNAct(in_channels, hid, 1, act_type=act_type)
        for i, d in enumerate(self.DILATIONS, start=2):
            setattr(self, f"stage{i}", ConvBNAct(in_channels, hid, 3, dilation=d, act_type=act_type))
        self.stage5 = nn.Sequential(nn.AdaptiveAvgPool2d(1), conv1x1(in_channels, in_channels - hid * 4))
        self.conv = ConvBNAct(2 * in_channels, out_channels, 1, act_type=act_type)

    def forward(self, x):
        branches = [x] + [getattr(self, f"stage{i}")(x) for i in range(1, 5)]
        branches.append(ops.interpolate(self.stage5(x), x.shape[2:], True))
        return self.conv(torch.cat(branches, dim=1))


class SegHead(nn.Sequential):
    def __init__(self, in_channels, num_class, act_type, hid_channels=256):
        super().__init__(ConvBNAct(in_channels, hid_channels, 3, act_type=act_type),
                         ConvBNAct(hid_channels, hid_channels // 2, 3, act_type=act_type),
                         conv1x1(hid_channels // 2, num_class))
