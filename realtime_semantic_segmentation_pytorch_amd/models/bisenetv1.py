"""BiSeNet V1 (arXiv:1808.00897).

Parity target: reference models/bisenetv1.py (BiSeNetv1 :16-32, SpatialPath
:35-41, ContextPath :44-73, AttentionRefinementModule :76-88,
FeatureFusionModule :91-114).  ARM/FFM evaluate their attention branch on the
pooled vector (``modules.pooled_conv_bn_act``) instead of on an ``expand_as``
copy of it -- same values and gradients, H*W times less work.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .backbone import ResNet
from .modules import ConvBNAct, SegHead, conv1x1, pooled_conv_bn_act


class BiSeNetv1(nn.Module):
    def __init__(self, num_class=1, n_channel=3, backbone_type="resnet18", act_type="relu",
                 pretrained=False):
        super().__init__()
        self.spatial_path = SpatialPath(n_channel, 128, act_type=act_type)
        self.context_path = ContextPath(256, backbone_type, act_type=act_type, pretrained=pretrained)
        self.ffm = FeatureFusionModule(384, 256, act_type=act_type)
        self.seg_head = SegHead(256, num_class, act_type=act_type)

    def forward(self, x, is_training=False):
        out_hw = x.shape[2:]
        x = self.seg_head(self.ffm(self.spatial_path(x), self.context_path(x)))
        return ops.final_upsample(x, out_hw, True)


class SpatialPath(nn.Sequential):
    def __init__(self, in_channels, out_channels, act_type):
        super().__init__(*[ConvBNAct(in_channels if i == 0 else out_channels, out_channels, 3, 2,
                                     act_type=act_type) for i in range(3)])


class ContextPath(nn.Module):
    def __init__(self, out_channels, backbone_type, act_type, pretrained=False):
        super().__init__()
        if "resnet" not in backbone_type:
            raise NotImplementedError()
        self.backbone = ResNet(backbone_type, pretrained=pretrained)
        c16, c32 = self.backbone.out_channels[2], self.backbone.out_channels[3]
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.arm_16 = AttentionRefinementModule(c16)
        self.arm_32 = AttentionRefinementModule(c32)
        self.conv_16 = conv1x1(c16, out_channels)
        self.conv_32 = conv1x1(c32, out_channels)

    def forward(self, x):
        _, _, x16, x32 = self.backbone(x)
        x32 = self.conv_32(self.arm_32(x32) + self.pool(x32))
        up = (x32.shape[2] * 2, x32.shape[3] * 2)
        x16 = ops.interpolate(x32, up, True, skip=self.conv_16(self.arm_16(x16)))
        return ops.interpolate(x16, (x16.shape[2] * 2, x16.shape[3] * 2), True)


class AttentionRefinementModule(nn.Module):
    def __init__(self, channels):
        super().__init__()
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.conv = ConvBNAct(channels, channels, 1, act_type="sigmoid")

    def forward(self, x):
        att = pooled_conv_bn_act(self.conv, self.pool(x), x.shape[2] * x.shape[3])
        return ops.gate(x, att)


class FeatureFusionModule(nn.Module):
    def __init__(self, in_channels, out_channels, act_type):
        super().__init__()
        self.conv1 = ConvBNAct(in_channels, out_channels, 3, act_type=act_type)
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.conv2 = nn.Sequential(conv1x1(out_channels, out_channels), nn.ReLU(),
                                   conv1x1(out_channels, out_channels), nn.Sigmoid())

    def forward(self, x_low, x_high):
        x = self.conv1(torch.cat([x_low, x_high], dim=1))
        att = self.conv2(self.pool(x))  # per-channel gate; broadcast == reference expand_as
        return ops.gate(x, att, mode="residual")  # x + x * att in one pass
