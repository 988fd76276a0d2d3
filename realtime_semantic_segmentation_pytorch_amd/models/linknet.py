"""LinkNet (arXiv:1707.03718).

Parity target: reference models/linknet.py (LinkNet :15-38, DecoderBlock
:41-57, SegHead :60-67).  The ResNet encoder features are added into the
decoder path ("links"); the head's two transposed convs restore full
resolution, so the model output needs no final resize.
"""
from __future__ import annotations

import torch.nn as nn

from .backbone import ResNet
from .modules import ConvBNAct, DeConvBNAct


class LinkNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, backbone_type="resnet18", act_type="relu",
                 pretrained=False):
        super().__init__()
        if "resnet" not in backbone_type:
            raise NotImplementedError()
        self.backbone = ResNet(backbone_type, pretrained=pretrained)
        c = self.backbone.out_channels
        self.dec_block4 = DecoderBlock(c[3], c[2], act_type)
        self.dec_block3 = DecoderBlock(c[2], c[1], act_type)
        self.dec_block2 = DecoderBlock(c[1], c[0], act_type)
        self.dec_block1 = DecoderBlock(c[0], c[0], act_type, scale_factor=1)
        self.seg_head = SegHead(c[0], num_class, act_type)

    def forward(self, x, is_training=False):
        f1, f2, f3, f4 = self.backbone(x)
        y = self.dec_block4(f4)
        for skip, block in ((f3, self.dec_block3), (f2, self.dec_block2), (f1, self.dec_block1)):
            y = block(y + skip)
        return self.seg_head(y)


class DecoderBlock(nn.Module):
    """1x1 (C/4) -> transposed conv x`scale_factor` (or 3x3) -> 1x1."""

    def __init__(self, in_channels, out_channels, act_type, scale_factor=2):
        super().__init__()
        hid = in_channels // 4
        self.conv1 = ConvBNAct(in_channels, hid, 1, act_type=act_type)
        self.full_conv = (DeConvBNAct(hid, hid, scale_factor, act_type=act_type) if scale_factor > 1
                          else ConvBNAct(hid, hid, 3, act_type=act_type))
        self.conv2 = ConvBNAct(hid, out_channels, 1, act_type=act_type)

    def forward(self, x):
        return self.conv2(self.full_conv(self.conv1(x)))


class SegHead(nn.Sequential):
    def __init__(self, in_channels, num_class, act_type, scale_factor=2):
        hid = in_channels // 2
        super().__init__(DeConvBNAct(in_channels, hid, scale_factor, act_type=act_type),
                         ConvBNAct(hid, hid, 3, act_type=act_type),
                         DeConvBNAct(hid, num_class, scale_factor, act_type=act_type))
