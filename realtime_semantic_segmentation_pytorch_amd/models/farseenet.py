"""FarSee-Net (arXiv:2003.03913).

Parity target: reference models/farseenet.py (FarSeeNet :17-38, FASPP :41-106:
factorized ASPP on the 1/32 features with sub-pixel (PixelShuffle x2) fusion
into the 1/16 features, then a x4 sub-pixel classifier).  Key names match
(``frontend_network`` / ``backend_network``).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .backbone import ResNet
from .modules import ConvBNAct, DWConvBNAct, conv1x1


class FarSeeNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, backbone_type="resnet18", act_type="relu",
                 pretrained=False):
        super().__init__()
        if "resnet" not in backbone_type:
            raise NotImplementedError()
        self.frontend_network = ResNet(backbone_type, pretrained=pretrained)
        c = self.frontend_network.out_channels
        self.backend_network = FASPP(c[3], c[2], num_class, act_type)

    def forward(self, x, is_training=False):
        _, _, x16, x32 = self.frontend_network(x)
        return ops.final_upsample(self.backend_network(x32, x16), x.shape[2:], True)


def _factorized(cin, cout, dilation, act_type):
    """1x1 reduction followed by a dilated depth-wise 3x3."""
    return nn.Sequential(ConvBNAct(cin, cout, 1, act_type=act_type),
                         DWConvBNAct(cout, cout, 3, dilation=dilation, act_type=act_type))


class FASPP(nn.Module):
    def __init__(self, high_channels, low_channels, num_class, act_type, dilations=(6, 12, 18),
                 hid_channels=256):
        super().__init__()
        h = hid_channels
        self.conv_high = nn.ModuleList([ConvBNAct(high_channels, h, 1, act_type=act_type)] +
                                       [_factorized(high_channels, h, d, act_type) for d in dilations])
        self.sub_pixel_high = nn.Sequential(conv1x1(h * 4, h * 2 * 4), nn.PixelShuffle(2))
        self.conv_low_init = ConvBNAct(low_channels, 48, 1, act_type=act_type)
        self.conv_low = nn.ModuleList([ConvBNAct(h * 2 + 48, h // 2, 1, act_type=act_type)] +
                                      [_factorized(h * 2 + 48, h // 2, d, act_type) for d in dilations[:-1]])
        self.conv_low_last = nn.Sequential(ConvBNAct(h // 2 * 3, h * 2, 1, act_type=act_type),
                                           ConvBNAct(h * 2, h * 2, act_type=act_type))
        self.sub_pixel_low = nn.Sequential(conv1x1(h * 2, num_class * 16), nn.PixelShuffle(4))

    def forward(self, x_high, x_low):
        y = self.sub_pixel_high(torch.cat([m(x_high) for m in self.conv_high], dim=1))
        y = torch.cat([y, self.conv_low_init(x_low)], dim=1)
        y = self.conv_low_last(torch.cat([m(y) for m in self.conv_low], dim=1))
        return self.sub_pixel_low(y)
