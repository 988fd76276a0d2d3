"""RegSeg (arXiv:2111.09957) -- rethinking dilated convolution (D-blocks).

Parity target: reference models/regseg.py (RegSeg :15-59, DBlock :62-110 --
1x1, split into two grouped 3x3 convs of different dilation (stride 1) or a
grouped strided 3x3 with avg-pool shortcut (stride 2), SE, 1x1, residual;
SEBlock :113-131, Decoder :134-167).  The reference's ConvBNAct has no
``groups`` argument, so reference RegSeg cannot be constructed (SURVEY A.1
#8); here ``groups`` is supported and the module tree / key names are what the
reference intends.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .modules import Activation, ConvBNAct, conv1x1

DEFAULT_DILATIONS = ((1, 1), (1, 2), (1, 2), (1, 3), (2, 3), (2, 7), (2, 3), (2, 6), (2, 5), (2, 9), (2, 11),
                     (4, 7), (5, 14))


class RegSeg(nn.Module):
    def __init__(self, num_class=1, n_channel=3, dilations=None, act_type="relu"):
        super().__init__()
        if dilations is None:
            dilations = DEFAULT_DILATIONS
        elif len(dilations) != 13:
            raise ValueError("Dilation pairs' length should be 13\n")
        self.conv_init = ConvBNAct(n_channel, 32, 3, 2, act_type=act_type)
        self.stage_d4 = DBlock(32, 48, 2, act_type=act_type)
        self.stage_d8 = nn.Sequential(DBlock(48, 128, 2, act_type=act_type),
                                      *[DBlock(128, 128, 1, r1=1, r2=1, act_type=act_type) for _ in range(2)])
        d16 = [DBlock(128, 256, 2, act_type=act_type)]
        d16 += [DBlock(256, 256, 1, r1=a, r2=b, act_type=act_type) for a, b in dilations[:12]]
        d16.append(DBlock(256, 320, 2, r1=dilations[-1][0], r2=dilations[-1][1], act_type=act_type))
        self.stage_d16 = nn.Sequential(*d16)
        self.decoder = Decoder(num_class, 48, 128, 320, act_type)

    def forward(self, x, is_training=False):
        d4 = self.stage_d4(self.conv_init(x))
        d8 = self.stage_d8(d4)
        d16 = self.stage_d16(d8)
        return ops.final_upsample(self.decoder(d4, d8, d16), x.shape[2:], True)


class DBlock(nn.Module):
    def __init__(self, in_channels, out_channels, stride=1, r1=None, r2=None, g=16, se_ratio=0.25, act_type="relu"):
        super().__init__()
        if stride not in (1, 2):
            raise AssertionError(f"Unsupported stride: {stride}")
        self.stride = stride
        self.conv1 = ConvBNAct(in_channels, out_channels, 1, act_type=act_type)
        if stride == 1:
            if in_channels != out_channels:
                raise AssertionError("In_channels should be the same as out_channels when stride = 1")
            split = out_channels // 2
            if split % g:
                raise AssertionError("Group width `g` should be evenly divided by split_ch")
            self.split_channels = split
            self.conv_left = ConvBNAct(split, split, 3, dilation=r1, groups=split // g, act_type=act_type)
            self.conv_right = ConvBNAct(split, split, 3, dilation=r2, groups=split // g, act_type=act_type)
        else:
            if out_channels % g:
                raise AssertionError("Group width `g` should be evenly divided by out_channels")
            self.conv_left = ConvBNAct(out_channels, out_channels, 3, 2, groups=out_channels // g, act_type=act_type)
            self.conv_skip = nn.Sequential(nn.AvgPool2d(2, 2, 0), ConvBNAct(in_channels, out_channels, 1, act_type="none"))
        self.conv2 = nn.Sequential(SEBlock(out_channels, se_ratio, act_type),
                                   ConvBNAct(out_channels, out_channels, 1, act_type="none"))
        self.act = Activation(act_type)

    def forward(self, x):
        h = self.conv1(x)
        if self.stride == 1:
            s = self.split_channels
            h = torch.cat([self.conv_left(h[:, :s]), self.conv_right(h[:, s:])], dim=1)
            res = x
        else:
            h = self.conv_left(h)
            res = self.conv_skip(x)
        return self.conv2[1](self.conv2[0](h), residual=res, act=self.act)


class SEBlock(nn.Module):
    def __init__(self, channels, reduction_ratio, act_type):
        super().__init__()
        sq = int(channels * reduction_ratio)
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.se_block = nn.Sequential(nn.Linear(channels, sq), Activation(act_type), nn.Linear(sq, channels),
                                      Activation("sigmoid"))

    def forward(self, x):
        w = self.se_block(x.mean(dim=(2, 3)))
        return ops.gate(x, w[:, :, None, None])


class Decoder(nn.Module):
    def __init__(self, num_class, d4_channel, d8_channel, d16_channel, act_type):
        super().__init__()
        self.conv_d16 = ConvBNAct(d16_channel, 128, 1, act_type=act_type)
        self.conv_d8_stage1 = ConvBNAct(d8_channel, 128, 1, act_type=act_type)
        self.conv_d4_stage1 = ConvBNAct(d4_channel, 8, 1, act_type=act_type)
        self.conv_d8_stage2 = ConvBNAct(128, 64, 3, act_type=act_type)
        self.conv_d4_stage2 = nn.Sequential(ConvBNAct(64 + 8, 64, 3, act_type=act_type), conv1x1(64, num_class))

    def forward(self, x_d4, x_d8, x_d16):
        y8 = ops.interpolate(self.conv_d16(x_d16), x_d8.shape[2:], True, skip=self.conv_d8_stage1(x_d8))
        y4 = ops.interpolate(self.conv_d8_stage2(y8), x_d4.shape[2:], True)
        return self.conv_d4_stage2(torch.cat([self.conv_d4_stage1(x_d4), y4], dim=1))
