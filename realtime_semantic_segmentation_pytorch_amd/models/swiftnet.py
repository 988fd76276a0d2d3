"""SwiftNet (arXiv:1903.08469).

Parity target: reference models/swiftnet.py (SwiftNet :17-49 with ResNet or
MobileNetV2 backbone, SPP = PyramidPoolingModule, Decoder :52-72 -- a ladder of
"upsample x2 + lateral add + 3x3 ConvBNAct").  Each ladder rung's
upsample-and-add is one fused resize-add kernel.
"""
from __future__ import annotations

import torch.nn as nn

from .. import ops
from .backbone import Mobilenetv2, ResNet
from .modules import ConvBNAct, PyramidPoolingModule


def make_backbone(backbone_type, pretrained=False):
    """(backbone, stage channels) for the reference's backbone names."""
    if "resnet" in backbone_type:
        bb = ResNet(backbone_type, pretrained=pretrained)
        return bb, bb.out_channels
    if backbone_type == "mobilenet_v2":
        bb = Mobilenetv2(pretrained=pretrained)
        return bb, bb.out_channels
    raise NotImplementedError()


class SwiftNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, backbone_type="resnet18", up_channels=128,
                 act_type="relu", pretrained=False):
        super().__init__()
        self.backbone, ch = make_backbone(backbone_type, pretrained)
        for i in range(3):
            setattr(self, f"connection{i + 1}", ConvBNAct(ch[i], up_channels, 1, act_type=act_type))
        self.spp = PyramidPoolingModule(ch[3], up_channels, act_type, bias=True)
        self.decoder = Decoder(up_channels, num_class, act_type)

    def forward(self, x, is_training=False):
        x1, x2, x3, x4 = self.backbone(x)
        lat = (self.connection1(x1), self.connection2(x2), self.connection3(x3))
        y = self.decoder(self.spp(x4), *lat)
        return ops.final_upsample(y, x.shape[2:], True)


class Decoder(nn.Module):
    def __init__(self, channels, num_class, act_type):
        super().__init__()
        self.up_stage3 = ConvBNAct(channels, channels, 3, act_type=act_type)
        self.up_stage2 = ConvBNAct(channels, channels, 3, act_type=act_type)
        self.up_stage1 = ConvBNAct(channels, num_class, 3, act_type=act_type)

    def forward(self, x, x1, x2, x3):
        for lateral, stage in ((x3, self.up_stage3), (x2, self.up_stage2), (x1, self.up_stage1)):
            x = stage(ops.interpolate(x, (x.shape[2] * 2, x.shape[3] * 2), True, skip=lateral))
        return x
