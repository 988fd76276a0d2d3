"""LEDNet (arXiv:1905.02423) -- split-shuffle non-bottleneck encoder + attention pyramid decoder.

Parity target: reference models/lednet.py (LEDNet :16-27, Encoder :30-50,
SSnbtUnit :53-93 -- channel split, two factorized branches, residual, act,
channel shuffle; AttentionPyramidNetwork :96-150).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .enet import InitialBlock as DownsampleUint
from .modules import Activation, ConvBNAct, channel_shuffle

_ENCODER_PLAN = ((32, (1, 1, 1)), (64, (1, 1)), (None, (1, 2, 5, 9, 2, 5, 9, 17)))


class LEDNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="relu"):
        super().__init__()
        self.encoder = Encoder(n_channel, 128, act_type)
        self.apn = AttentionPyramidNetwork(128, num_class, act_type)

    def forward(self, x, is_training=False):
        return ops.final_upsample(self.apn(self.encoder(x)), x.shape[2:], True)


class Encoder(nn.Sequential):
    def __init__(self, in_channels, out_channels, act_type):
        mods, cin = [], in_channels
        for cout, dils in _ENCODER_PLAN:
            cout = out_channels if cout is None else cout
            mods.append(DownsampleUint(cin, cout, act_type))
            mods += [SSnbtUnit(cout, d, act_type=act_type) for d in dils]
            cin = cout
        super().__init__(*mods)


def _factorized_branch(ch, first, second, dilation, act_type):
    """conv(first)+bias -> act -> ConvBNAct(second) -> dilated conv(first)+bias -> act -> dilated ConvBNAct(second)."""
    def pad(k, d):
        return tuple((kk - 1) // 2 * d for kk in k)
    return nn.Sequential(
        nn.Conv2d(ch, ch, first, padding=pad(first, 1)), Activation(act_type),
        ConvBNAct(ch, ch, second, act_type=act_type),
        nn.Conv2d(ch, ch, first, padding=pad(first, dilation), dilation=dilation), Activation(act_type),
        ConvBNAct(ch, ch, second, dilation=dilation, act_type=act_type))


class SSnbtUnit(nn.Module):
    def __init__(self, channels, dilation, act_type):
        super().__init__()
        if channels % 2:
            raise AssertionError("Input channel should be multiple of 2.\n")
        h = channels // 2
        self.split_channels = h
        self.left_branch = _factorized_branch(h, (3, 1), (1, 3), dilation, act_type)
        self.right_branch = _factorized_branch(h, (1, 3), (3, 1), dilation, act_type)
        self.act = Activation(act_type)

    def forward(self, x):
        h = self.split_channels
        y = torch.cat([self.left_branch(x[:, :h]), self.right_branch(x[:, h:])], dim=1)
        return channel_shuffle(self.act(x + y))


class AttentionPyramidNetwork(nn.Module):
    def __init__(self, in_channels, out_channels, act_type):
        super().__init__()
        c, o = in_channels, out_channels
        self.left_conv1_1 = ConvBNAct(c, c, 3, 2, act_type=act_type)
        self.left_conv1_2 = ConvBNAct(c, o, 3, act_type=act_type)
        self.left_conv2_1 = ConvBNAct(c, c, 3, 2, act_type=act_type)
        self.left_conv2_2 = ConvBNAct(c, o, 3, act_type=act_type)
        self.left_conv3 = nn.Sequential(ConvBNAct(c, c, 3, 2, act_type=act_type),
                                        ConvBNAct(c, o, 3, act_type=act_type))
        self.mid_branch = ConvBNAct(c, o, act_type=act_type)
        self.right_branch = nn.Sequential(nn.AdaptiveAvgPool2d(1), ConvBNAct(c, o, act_type=act_type))

    def forward(self, x):
        l1 = self.left_conv1_1(x)
        l2 = self.left_conv2_1(l1)
        l3 = self.left_conv3(l2)
        # pyramid top-down: resize-and-add fused into the interpolation kernel
        l2 = ops.interpolate(l3, l2.shape[2:], True, skip=self.left_conv2_2(l2))
        l1 = ops.interpolate(l2, l1.shape[2:], True, skip=self.left_conv1_2(l1))
        att = ops.interpolate(l1, x.shape[2:], True)
        g = self.right_branch(x)  # [N, o, 1, 1]: a bilinear resize of 1x1 is a broadcast
        return att * self.mid_branch(x) + g
