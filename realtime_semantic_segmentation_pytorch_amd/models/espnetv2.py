"""ESPNetv2 (arXiv:1811.11431) -- extremely efficient spatial pyramid (EESP) units.

Parity target: reference models/espnetv2.py (ESPNetv2 :16-54 with pooled
image injection into strided units, build_blocks :57-61, EESPModule :64-116 --
grouped 1x1 reduce, K depth-wise dilated branches, hierarchical sum, grouped
1x1 expand, residual or pooled-concat + image shortcut).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .modules import ConvBNAct, DSConvBNAct, PyramidPoolingModule, SegHead, conv1x1


class ESPNetv2(nn.Module):
    def __init__(self, num_class=1, n_channel=3, K=4, alpha3=3, alpha4=7, act_type="prelu"):
        super().__init__()
        self.pool = nn.AvgPool2d(3, 2, 1)
        self.l1_block = ConvBNAct(n_channel, 32, 3, 2, act_type=act_type)
        self.l2_block = EESPModule(32, stride=2, act_type=act_type)
        self.l3_block1 = EESPModule(64, stride=2, act_type=act_type)
        self.l3_block2 = build_blocks(EESPModule, 128, alpha3, act_type=act_type)
        self.l4_block1 = EESPModule(128, stride=2, act_type=act_type)
        self.l4_block2 = build_blocks(EESPModule, 256, alpha4, act_type=act_type)
        self.convl4_l3 = ConvBNAct(256, 128, 1)
        self.ppm = PyramidPoolingModule(256, 256, act_type=act_type, bias=True)
        self.decoder = SegHead(256, num_class, act_type=act_type)

    def forward(self, x, is_training=False):
        d4 = self.pool(self.pool(x))
        d8 = self.pool(d4)
        d16 = self.pool(d8)
        y = self.l2_block(self.l1_block(x), d4)
        x3 = self.l3_block2(self.l3_block1(y, d8))
        y = self.l4_block2(self.l4_block1(x3, d16))
        y = self.convl4_l3(ops.interpolate(y, x3.shape[2:], True))
        y = self.decoder(self.ppm(torch.cat([y, x3], dim=1)))
        return ops.final_upsample(y, x.shape[2:], True)


def build_blocks(block, channels, num_block, act_type="relu"):
    return nn.Sequential(*[block(channels, act_type=act_type) for _ in range(num_block)])


class EESPModule(nn.Module):
    def __init__(self, channels, K=4, ks=3, stride=1, act_type="prelu"):
        super().__init__()
        if channels % K:
            raise AssertionError("Input channels should be integer multiples of K.\n")
        self.K = K
        ck = channels // K
        self.use_skip = stride == 1
        self.conv_init = nn.Conv2d(channels, ck, 1, groups=K, bias=False)
        self.layers = nn.ModuleList([DSConvBNAct(ck, ck, ks, stride, 2 ** k, act_type=act_type) for k in range(K)])
        self.conv_last = nn.Conv2d(channels, channels, 1, groups=K, bias=False)
        if not self.use_skip:
            self.pool = nn.AvgPool2d(3, 2, 1)
            self.conv_stride = nn.Sequential(ConvBNAct(3, 3, 3), conv1x1(3, channels * 2))

    def forward(self, x, img=None):
        if not self.use_skip and img is None:
            raise ValueError("Strided EESP unit needs downsampled input image.\n")
        r = self.conv_init(x)
        feats, run = [], None
        for layer in self.layers:
            f = layer(r)
            run = f if run is None else f + run
            feats.append(run)
        y = self.conv_last(torch.cat(feats, dim=1))
        if self.use_skip:
            return y + x
        return torch.cat([y, self.pool(x)], dim=1) + self.conv_stride(img)
