"""CANet -- Cross Attention Network for semantic segmentation (arXiv:1907.10958).

Parity target: reference models/canet.py (CANet :15-30, SpatialBranch :33-39,
ContextBranch :42-65, FeatureCrossAttentionModule :68-89, spatial / channel
attention :92-117).  The two attention maps are combined into one broadcast
gate before touching the full feature map; the x8 transposed-conv head gives
full-resolution logits directly.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .backbone import Mobilenetv2, ResNet
from .modules import ConvBNAct, DeConvBNAct


class CANet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, backbone_type="mobilenet_v2", act_type="relu",
                 pretrained=False):
        super().__init__()
        self.spatial_branch = SpatialBranch(n_channel, 64, act_type)
        self.context_branch = ContextBranch(64 * 4, backbone_type, pretrained=pretrained)
        self.fca = FeatureCrossAttentionModule(64 * 4, num_class, act_type)
        self.up = DeConvBNAct(num_class, num_class, scale_factor=8)

    def forward(self, x, is_training=False):
        return self.up(self.fca(self.spatial_branch(x), self.context_branch(x)))


class SpatialBranch(nn.Sequential):
    def __init__(self, n_channel, channels, act_type):
        widths = (n_channel, channels, channels * 2, channels * 4)
        super().__init__(*[ConvBNAct(widths[i], widths[i + 1], 3, 2, act_type=act_type, inplace=True)
                           for i in range(3)])


class ContextBranch(nn.Module):
    def __init__(self, out_channels, backbone_type, hid_channels=192, pretrained=False):
        super().__init__()
        if "mobilenet" in backbone_type:
            self.backbone = Mobilenetv2(pretrained=pretrained)
        elif "resnet" in backbone_type:
            self.backbone = ResNet(backbone_type, pretrained=pretrained)
        else:
            raise NotImplementedError()
        c32, c16 = self.backbone.out_channels[3], self.backbone.out_channels[2]
        self.up1 = DeConvBNAct(c32, hid_channels)
        self.up2 = DeConvBNAct(c16 + hid_channels, out_channels)

    def forward(self, x):
        _, _, x16, x32 = self.backbone(x)
        return self.up2(torch.cat([self.up1(x32), x16], dim=1))


class FeatureCrossAttentionModule(nn.Module):
    def __init__(self, in_channels, out_channels, act_type):
        super().__init__()
        self.conv_init = ConvBNAct(2 * in_channels, in_channels, act_type=act_type, inplace=True)
        self.sa = SpatialAttentionBlock(in_channels)
        self.ca = ChannelAttentionBlock(in_channels)
        self.conv_last = ConvBNAct(in_channels, out_channels, inplace=True)

    def forward(self, x_s, x_c):
        fused = self.conv_init(torch.cat([x_s, x_c], dim=1))
        gate = self.sa(x_s) * self.ca(x_c)  # [N,1,H,W] * [N,C,1,1]
        return self.conv_last(ops.gate(fused, gate, mode="residual"))  # fused * gate + fused


class SpatialAttentionBlock(nn.Sequential):
    def __init__(self, in_channels):
        super().__init__(ConvBNAct(in_channels, 1, act_type="sigmoid"))


class ChannelAttentionBlock(nn.Module):
    """Shared FC over global max- and average-pooled descriptors, summed, sigmoid."""

    def __init__(self, in_channels):
        super().__init__()
        self.in_channels = in_channels
        self.max_pool = nn.AdaptiveMaxPool2d(1)
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(in_channels, in_channels)

    def forward(self, x):
        d_max = self.fc(self.max_pool(x).flatten(1))
        d_avg = self.fc(self.avg_pool(x).flatten(1))
        return torch.sigmoid(d_max + d_avg)[:, :, None, None]
