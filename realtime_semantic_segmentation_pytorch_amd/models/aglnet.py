"""AGLNet (Applied Soft Computing 2020) -- attention-guided lightweight network.

Parity target: reference models/aglnet.py (AGLNet :17-56 reusing ENet's
initial block and LEDNet's SSnbtUnit, FAPM :72-94, PyramidFeatureAttention
:97-130, GAUM :133-157, spatial / channel attention :160-179).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .enet import InitialBlock as DownsamplingUnit
from .lednet import SSnbtUnit
from .modules import Activation, ConvBNAct, conv1x1


def build_blocks(block, channels, num_block, dilations=(), act_type="relu"):
    dilations = list(dilations) or [1] * num_block
    if len(dilations) != num_block:
        raise ValueError("Number of dilation should be equal to number of blocks")
    return nn.Sequential(*[block(channels, dilation=d, act_type=act_type) for d in dilations])


class AGLNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="relu"):
        super().__init__()
        self.layer1 = DownsamplingUnit(n_channel, 32, act_type=act_type)
        self.layer2_4 = build_blocks(SSnbtUnit, 32, 3, act_type=act_type)
        self.layer5 = DownsamplingUnit(32, 64, act_type=act_type)
        self.layer6_7 = build_blocks(SSnbtUnit, 64, 2, act_type=act_type)
        self.layer8 = DownsamplingUnit(64, 128, act_type=act_type)
        self.layer9_16 = build_blocks(SSnbtUnit, 128, 8, dilations=(1, 2, 5, 9, 2, 5, 9, 17), act_type=act_type)
        self.layer17 = FAPM(128, act_type=act_type)
        self.layer18 = GAUM(64, 128, 64, act_type=act_type)
        self.layer19 = GAUM(32, 64, 32, act_type=act_type)
        self.layer20 = conv1x1(32, num_class)

    def forward(self, x, is_training=False):
        s1 = self.layer2_4(self.layer1(x))
        s2 = self.layer6_7(self.layer5(s1))
        y = self.layer17(self.layer9_16(self.layer8(s2)))
        y = self.layer19(self.layer18(y, s2), s1)
        return ops.final_upsample(self.layer20(y), x.shape[2:], True)


class FAPM(nn.Module):
    """Feature attention pyramid: x * conv(pyramid_attention(x)) + global context."""

    def __init__(self, channels, act_type):
        super().__init__()
        self.pfa = PyramidFeatureAttention(channels, act_type)
        self.conv = conv1x1(1, channels)
        self.gp = nn.Sequential(nn.AdaptiveAvgPool2d(1), conv1x1(channels, channels))

    def forward(self, x):
        return x * self.conv(self.pfa(x)) + self.gp(x)  # resize of a 1x1 map == broadcast


class PyramidFeatureAttention(nn.Module):
    def __init__(self, channels, act_type):
        super().__init__()
        for i, k in enumerate((7, 5, 3), start=1):
            cin = channels if i == 1 else 1
            setattr(self, f"conv{i}1", ConvBNAct(cin, 1, (1, k), 2, act_type=act_type))
            setattr(self, f"conv{i}2", ConvBNAct(1, 1, (k, 1), 1, act_type=act_type))

    def forward(self, x):
        d1 = self.conv11(x)
        d2 = self.conv21(d1)
        d3 = self.conv32(self.conv31(d2))
        y = ops.interpolate(d3, d2.shape[2:], True, skip=self.conv22(d2))
        y = ops.interpolate(y, d1.shape[2:], True, skip=self.conv12(d1))
        return ops.interpolate(y, x.shape[2:], True)


class GAUM(nn.Module):
    """Global attention upsample: deconv(high) gated by spatial (low) and channel attention."""

    def __init__(self, low_channels, high_channels, out_channels, act_type):
        super().__init__()
        self.up_conv = nn.Sequential(nn.ConvTranspose2d(high_channels, low_channels, 3, 2, 1, 1),
                                     nn.BatchNorm2d(low_channels), Activation(act_type))
        self.sab = SpatialAttentionBlock(low_channels)
        self.cab = ChannelAttentionBlock(low_channels, out_channels)

    def forward(self, x_high, x_low):
        x_low = self.sab(x_low)
        up = self.up_conv[0](x_high)
        up = ops.bn_act(up, self.up_conv[1], self.up_conv[2], act_module=self.up_conv[2])
        gated = up * x_low
        return self.cab(gated) * gated + up


class SpatialAttentionBlock(nn.Module):
    def __init__(self, channels):
        super().__init__()
        self.conv = conv1x1(channels, 1)

    def forward(self, x):
        return ops.gate(x, self.conv(x), sigmoid=True)


class ChannelAttentionBlock(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.conv = conv1x1(in_channels, out_channels)

    def forward(self, x):
        return ops.gate(x, self.conv(self.pool(x)), sigmoid=True)
