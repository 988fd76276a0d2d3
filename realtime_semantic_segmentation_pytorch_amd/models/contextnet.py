"""ContextNet (arXiv:1805.04554) -- full-resolution detail branch + 1/4-input context branch.

Parity target: reference models/contextnet.py (ContextNet :15-33, Branch_1
:36-48, Branch_4 :51-82 (MobileNetV2 bottlenecks), FeatureFusion :85-109,
InvertedResidual :112-129 == Fast-SCNN's).
"""
from __future__ import annotations

import torch.nn as nn

from .. import ops
from .fastscnn import InvertedResidual, inverted_residual_stack  # noqa: F401  (same block)
from .modules import Activation, ConvBNAct, DSConvBNAct, DWConvBNAct, PWConvBNAct, conv1x1

BRANCH4_PLAN = ((1, 32, 1, 1), (6, 32, 1, 1), (6, 48, 3, 2), (6, 64, 3, 2), (6, 96, 2, 1), (6, 128, 2, 1))


class ContextNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="relu"):
        super().__init__()
        self.full_res_branch = Branch_1(n_channel, (32, 64, 128), 128, act_type=act_type)
        self.lower_res_branch = Branch_4(n_channel, 128, act_type=act_type)
        self.feature_fusion = FeatureFusion(128, 128, 128, act_type=act_type)
        self.classifier = ConvBNAct(128, num_class, 1, act_type=act_type)

    def forward(self, x, is_training=False):
        h, w = x.shape[2:]
        low = self.lower_res_branch(ops.interpolate(x, (h // 4, w // 4), True))
        y = self.classifier(self.feature_fusion(self.full_res_branch(x), low))
        return ops.final_upsample(y, (h, w), True)


class Branch_1(nn.Sequential):
    def __init__(self, in_channels, hid_channels, out_channels, act_type="relu"):
        if len(hid_channels) != 3:
            raise AssertionError
        c = list(hid_channels) + [out_channels]
        mods = [ConvBNAct(in_channels, c[0], 3, 2, act_type=act_type)]
        for a, b in zip(c[:3], c[1:]):
            mods += [DWConvBNAct(a, a, 3, 1, act_type="none"), PWConvBNAct(a, b, act_type=act_type)]
        super().__init__(*mods)


class Branch_4(nn.Module):
    def __init__(self, in_channels, out_channels, act_type="relu"):
        super().__init__()
        self.conv_init = ConvBNAct(in_channels, 32, 3, 2, act_type=act_type)
        self.bottlenecks, c = inverted_residual_stack(32, BRANCH4_PLAN, act_type)
        self.conv_last = ConvBNAct(c, out_channels, 3, 1, act_type=act_type)

    def forward(self, x):
        return self.conv_last(self.bottlenecks(self.conv_init(x)))


class FeatureFusion(nn.Module):
    def __init__(self, branch_1_channels, branch_4_channels, out_channels, act_type="relu"):
        super().__init__()
        self.branch_1_conv = conv1x1(branch_1_channels, out_channels)
        self.branch_4_conv = nn.Sequential(
            DSConvBNAct(branch_4_channels, out_channels, 3, dilation=4, act_type="none"),
            conv1x1(out_channels, out_channels))
        self.act = Activation(act_type=act_type)

    def forward(self, f1, f4):
        f4 = self.branch_4_conv(ops.interpolate(f4, f1.shape[2:], True))
        return self.act(self.branch_1_conv(f1) + f4)
