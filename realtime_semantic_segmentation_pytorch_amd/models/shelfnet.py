"""ShelfNet (arXiv:1811.11254).

Parity target: reference models/shelfnet.py (ShelfNet :16-59 -- four "shelf"
columns over ResNet features: 1x1 lateral convs, decoder, encoder, decoder;
EncoderBlock :62-84, DecoderBlock :87-116, SBlock :119-135, a residual 3x3 pair
taking the lateral and vertical inputs).  SBlock's ``act(conv2(.) + residual)``
is one fused BN/residual/activation kernel.
"""
from __future__ import annotations

import torch.nn as nn

from .. import ops
from .backbone import ResNet
from .modules import Activation, ConvBNAct, DeConvBNAct, conv1x1


class ShelfNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, backbone_type="resnet18", hid_channels=(32, 64, 128, 256),
                 act_type="relu", pretrained=False):
        super().__init__()
        if "resnet" not in backbone_type:
            raise NotImplementedError()
        self.backbone = ResNet(backbone_type, pretrained=pretrained)
        c, h = self.backbone.out_channels, list(hid_channels)
        for i, tag in enumerate("ABCD"):
            setattr(self, f"conv_{tag}", ConvBNAct(c[i], h[i], 1, act_type=act_type))
        self.decoder2 = DecoderBlock(h, act_type)
        self.encoder3 = EncoderBlock(h, act_type)
        self.decoder4 = DecoderBlock(h, act_type)
        self.classifier = conv1x1(h[0], num_class)

    def forward(self, x, is_training=False):
        feats = self.backbone(x)
        cols = [getattr(self, f"conv_{t}")(f) for t, f in zip("ABCD", feats)]   # column 1
        a, b, c = self.decoder2(*cols, return_hid_feats=True)                     # column 2
        a, b, c, d = self.encoder3(a, b, c)                                        # column 3
        y = self.classifier(self.decoder4(a, b, c, d))                             # column 4
        return ops.final_upsample(y, x.shape[2:], True)


class EncoderBlock(nn.Module):
    def __init__(self, channels, act_type):
        super().__init__()
        for i, tag in enumerate("ABC"):
            setattr(self, f"block_{tag}", SBlock(channels[i], act_type))
            setattr(self, f"down_{tag}", ConvBNAct(channels[i], channels[i + 1], 3, 2, act_type=act_type))

    def forward(self, x_a, x_b, x_c):
        a = self.block_A(x_a)
        b = self.block_B(x_b, self.down_A(a))
        c = self.block_C(x_c, self.down_B(b))
        return a, b, c, self.down_C(c)


class DecoderBlock(nn.Module):
    def __init__(self, channels, act_type):
        super().__init__()
        self.block_D = SBlock(channels[3], act_type)
        self.up_D = DeConvBNAct(channels[3], channels[2], act_type=act_type)
        self.block_C = SBlock(channels[2], act_type)
        self.up_C = DeConvBNAct(channels[2], channels[1], act_type=act_type)
        self.block_B = SBlock(channels[1], act_type)
        self.up_B = DeConvBNAct(channels[1], channels[0], act_type=act_type)
        self.block_A = SBlock(channels[0], act_type)

    def forward(self, x_a, x_b, x_c, x_d, return_hid_feats=False):
        c = self.block_C(x_c, self.up_D(self.block_D(x_d)))
        b = self.block_B(x_b, self.up_C(c))
        a = self.block_A(x_a, self.up_B(b))
        return (a, b, c) if return_hid_feats else a


class SBlock(nn.Module):
    """act(conv2(conv1(l + v)) + (l + v)) -- lateral input l, vertical input v."""

    def __init__(self, channels, act_type):
        super().__init__()
        self.conv1 = ConvBNAct(channels, channels, 3, act_type=act_type)
        self.conv2 = ConvBNAct(channels, channels, 3, act_type="none")
        self.act = Activation(act_type)

    def forward(self, x_l, x_v=None):
        x = x_l if x_v is None else x_l + x_v
        return self.conv2(self.conv1(x), residual=x, act=self.act)
