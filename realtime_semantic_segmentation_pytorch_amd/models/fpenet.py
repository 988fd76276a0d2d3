"""FPENet (arXiv:1909.08599) -- feature pyramid encoding network.

Parity target: reference models/fpenet.py (FPENet :15-43, build_blocks
:46-50, FPEBlock :53-89 -- 1x1 expand, channel slices through depth-wise
convs of dilation 1/2/4/8 with hierarchical sum, 1x1 project, residual;
MEUModule :92-112 with spatial / channel attention :115-131).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .modules import ConvBNAct, DWConvBNAct


class FPENet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, p=3, q=9, k=4, act_type="relu"):
        super().__init__()
        self.stage1 = nn.Sequential(ConvBNAct(n_channel, 16, 3, 2, act_type=act_type, inplace=True),
                                    FPEBlock(16, 16, 1, 1, act_type=act_type))
        self.stage2_0 = FPEBlock(16, 32, k, 2, act_type=act_type)
        self.stage2 = build_blocks(FPEBlock, 32, p - 1, k, act_type)
        self.stage3_0 = FPEBlock(32, 64, k, 2, act_type=act_type)
        self.stage3 = build_blocks(FPEBlock, 64, q - 1, k, act_type)
        self.decoder2 = MEUModule(32, 64, 64, act_type)
        self.decoder1 = MEUModule(16, 64, 32, act_type)
        self.final = ConvBNAct(32, num_class, 1, act_type=act_type, inplace=True)

    def forward(self, x, is_training=False):
        x1 = self.stage1(x)
        x2 = self.stage2(self.stage2_0(x1))
        y = self.stage3(self.stage3_0(x2))
        y = self.final(self.decoder1(x1, self.decoder2(x2, y)))
        return ops.final_upsample(y, x.shape[2:], True)


def build_blocks(block, channels, num_block, expansion, act_type):
    return nn.Sequential(*[block(channels, channels, expansion, 1, act_type=act_type) for _ in range(num_block)])


class FPEBlock(nn.Module):
    def __init__(self, in_channels, out_channels, expansion, stride, dilations=(1, 2, 4, 8), act_type="relu"):
        super().__init__()
        if not dilations:
            raise AssertionError("Length of dilations should be larger than 0.\n")
        self.K = len(dilations)
        self.use_skip = in_channels == out_channels and stride == 1
        ce = out_channels * expansion
        self.ch = ce // self.K
        self.conv_init = ConvBNAct(in_channels, ce, 1, act_type=act_type, inplace=True)
        self.layers = nn.ModuleList([DWConvBNAct(self.ch, self.ch, 3, stride, d, act_type=act_type)
                                     for d in dilations])
        self.conv_last = ConvBNAct(ce, out_channels, 1, act_type=act_type)

    def forward(self, x):
        h = self.conv_init(x)
        feats, run = [], None
        for i, layer in enumerate(self.layers):
            f = layer(h[:, i * self.ch:(i + 1) * self.ch])
            run = f if run is None else f + run
            feats.append(run)
        y = self.conv_last(torch.cat(feats, dim=1))
        return y + x if self.use_skip else y


class MEUModule(nn.Module):
    """Mutual embedding upsample: low gated by channel attention(high), up(high) by spatial attention(low)."""

    def __init__(self, low_channels, high_channels, out_channels, act_type):
        super().__init__()
        self.conv_low = ConvBNAct(low_channels, out_channels, 1, act_type=act_type, inplace=True)
        self.conv_high = ConvBNAct(high_channels, out_channels, 1, act_type=act_type, inplace=True)
        self.sa = SpatialAttentionBlock(act_type)
        self.ca = ChannelAttentionBlock(out_channels, act_type)

    def forward(self, x_low, x_high):
        lo = self.conv_low(x_low)
        hi = self.conv_high(x_high)
        sa, ca = self.sa(lo), self.ca(hi)
        up = ops.interpolate(hi, (hi.shape[2] * 2, hi.shape[3] * 2), True)
        return lo * ca + up * sa


class SpatialAttentionBlock(nn.Module):
    def __init__(self, act_type):
        super().__init__()
        self.conv = ConvBNAct(1, 1, 1, act_type=act_type, inplace=True)

    def forward(self, x):
        return self.conv(x.mean(dim=1, keepdim=True))


class ChannelAttentionBlock(nn.Sequential):
    def __init__(self, channels, act_type):
        super().__init__(nn.AdaptiveAvgPool2d(1), ConvBNAct(channels, channels, 1, act_type=act_type, inplace=True))
