"""Fast-SCNN (arXiv:1902.04502).

Parity target: reference models/fastscnn.py (FastSCNN :16-32,
LearningToDownsample :35-41, GlobalFeatureExtractor :44-70 with MobileNetV2
inverted residuals + PPM, FeatureFusionModule :73-93, Classifier :96-102,
InvertedResidual :105-121).  Note the reference classifier ends in
PWConvBNAct *with* ReLU, i.e. non-negative logits; kept for parity.
"""
from __future__ import annotations

import torch.nn as nn

from .. import ops
from .modules import (Activation, ConvBNAct, DSConvBNAct, DWConvBNAct, PWConvBNAct,
                      PyramidPoolingModule, conv1x1)

# MobileNetV2 plan of the global feature extractor: (expand t, channels c, repeats n, stride s)
GFE_PLAN = ((6, 64, 3, 2), (6, 96, 2, 2), (6, 128, 3, 1))


class FastSCNN(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="relu"):
        super().__init__()
        self.learning_to_downsample = LearningToDownsample(n_channel, 64, act_type=act_type)
        self.global_feature_extractor = GlobalFeatureExtractor(64, 128, act_type=act_type)
        self.feature_fusion = FeatureFusionModule(64, 128, 128, act_type=act_type)
        self.classifier = Classifier(128, num_class, act_type=act_type)

    def forward(self, x, is_training=False):
        out_hw = x.shape[2:]
        hi = self.learning_to_downsample(x)
        x = self.classifier(self.feature_fusion(hi, self.global_feature_extractor(hi)))
        return ops.final_upsample(x, out_hw, True)


class LearningToDownsample(nn.Sequential):
    def __init__(self, in_channels, out_channels, hid_channels=(32, 48), act_type="relu"):
        c0, c1 = hid_channels
        super().__init__(ConvBNAct(in_channels, c0, 3, 2, act_type=act_type),
                         DSConvBNAct(c0, c1, 3, 2, act_type=act_type),
                         DSConvBNAct(c1, out_channels, 3, 2, act_type=act_type))


class InvertedResidual(nn.Module):
    """1x1 expand -> 3x3 depth-wise (stride) -> 1x1 linear projection (+ identity)."""

    def __init__(self, in_channels, out_channels, stride, expand_ratio=6, act_type="relu"):
        super().__init__()
        hid = int(round(in_channels * expand_ratio))
        self.use_res_connect = stride == 1 and in_channels == out_channels
        self.conv = nn.Sequential(PWConvBNAct(in_channels, hid, act_type=act_type),
                                  DWConvBNAct(hid, hid, 3, stride, act_type=act_type),
                                  ConvBNAct(hid, out_channels, 1, act_type="none"))

    def forward(self, x):
        h = self.conv[1](self.conv[0](x))
        return self.conv[2](h, residual=x if self.use_res_connect else None)


def inverted_residual_stack(cin, plan, act_type, block=InvertedResidual):
    layers = []
    for t, c, n, s in plan:
        for i in range(n):
            layers.append(block(cin, c, s if i == 0 else 1, t, act_type=act_type))
            cin = c
    return nn.Sequential(*layers), cin


class GlobalFeatureExtractor(nn.Module):
    def __init__(self, in_channels, out_channels, act_type="relu"):
        super().__init__()
        self.bottlenecks, c = inverted_residual_stack(in_channels, GFE_PLAN, act_type)
        self.ppm = PyramidPoolingModule(c, out_channels, act_type=act_type, bias=True)

    def forward(self, x):
        return self.ppm(self.bottlenecks(x))


class FeatureFusionModule(nn.Module):
    def __init__(self, higher_channels, lower_channels, out_channels, act_type="relu"):
        super().__init__()
        self.higher_res_conv = conv1x1(higher_channels, out_channels)
        self.lower_res_conv = nn.Sequential(DWConvBNAct(lower_channels, lower_channels, 3, 1, act_type=act_type),
                                            conv1x1(lower_channels, out_channels))
        self.non_linear = nn.Sequential(nn.BatchNorm2d(out_channels), Activation(act_type))

    def forward(self, higher, lower):
        lower = self.lower_res_conv(ops.interpolate(lower, higher.shape[2:], True))
        bn, act = self.non_linear[0], self.non_linear[1]
        return ops.bn_act(self.higher_res_conv(higher) + lower, bn, act, act_module=act)


class Classifier(nn.Sequential):
    def __init__(self, in_channels, num_class, act_type="relu"):
        super().__init__(DSConvBNAct(in_channels, in_channels, 3, 1, act_type=act_type),
                         DSConvBNAct(in_channels, in_channels, 3, 1, act_type=act_type),
                         PWConvBNAct(in_channels, num_class, act_type=act_type))
