"""PP-LiteSeg (arXiv:2204.02681).

Parity target: reference models/pp_liteseg.py (PPLiteSeg :15-32, Encoder
:35-47, SPPM :50-74, FLD :77-96, STDCBackbone :99-123, STDCModule :126-147,
UAFM :150-167, spatial / channel attention :170-201).  Key names match.
UAFM's ``alpha * up + (1 - alpha) * low`` blend is kept as a single fused
expression after a fused-capable resize; SPPM sums three resized pools.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .modules import ConvBNAct, conv1x1, conv3x3
from .stdc import STDC_REPEATS, STDCModule

DECODER_CHANNELS = {"stdc1": (32, 64, 128), "stdc2": (64, 96, 128)}


class PPLiteSeg(nn.Module):
    def __init__(self, num_class=1, n_channel=3, encoder_channels=(32, 64, 256, 512, 1024),
                 encoder_type="stdc1", fusion_type="spatial", act_type="relu"):
        super().__init__()
        enc = list(encoder_channels)
        dec = DECODER_CHANNELS[encoder_type]
        self.encoder = Encoder(n_channel, enc, encoder_type, act_type)
        self.sppm = SPPM(enc[-1], dec[0], act_type)
        self.decoder = FLD(enc, dec, num_class, fusion_type, act_type)

    def forward(self, x, is_training=False):
        x3, x4, x5 = self.encoder(x)
        return self.decoder(x3, x4, self.sppm(x5), x.shape[2:])


class Encoder(nn.Module):
    def __init__(self, in_channels, encoder_channels, encoder_type, act_type):
        super().__init__()
        if encoder_type not in STDC_REPEATS:
            raise ValueError(f"Unsupport encoder type: {encoder_type}.\n")
        self.encoder = STDCBackbone(in_channels, encoder_channels, encoder_type, act_type)

    def forward(self, x):
        return self.encoder(x)


class STDCBackbone(nn.Module):
    def __init__(self, in_channels, encoder_channels, encoder_type, act_type):
        super().__init__()
        reps = STDC_REPEATS[encoder_type]
        c = encoder_channels
        self.stage1 = ConvBNAct(in_channels, c[0], 3, 2)
        self.stage2 = ConvBNAct(c[0], c[1], 3, 2)
        for i, (cin, cout, n) in enumerate(zip(c[1:4], c[2:5], reps), start=3):
            setattr(self, f"stage{i}", nn.Sequential(STDCModule(cin, cout, 2, act_type),
                                                     *[STDCModule(cout, cout, 1, act_type) for _ in range(n)]))

    def forward(self, x):
        x3 = self.stage3(self.stage2(self.stage1(x)))
        x4 = self.stage4(x3)
        return x3, x4, self.stage5(x4)


class SPPM(nn.Module):
    """Simple pyramid pooling: 1x1 / 2x2 / 4x4 average pools -> ConvBNAct -> resize, summed, 3x3."""

    def __init__(self, in_channels, out_channels, act_type):
        super().__init__()
        hid = in_channels // 4
        self.act_type = act_type
        for i, ps in enumerate((1, 2, 4), start=1):
            setattr(self, f"pool{i}", nn.Sequential(nn.AdaptiveAvgPool2d(ps),
                                                    ConvBNAct(in_channels, hid, 1, act_type=act_type)))
        self.conv = conv3x3(hid, out_channels)

    def forward(self, x):
        hw = x.shape[2:]
        acc = ops.interpolate(self.pool1(x), hw, True)
        acc = ops.interpolate(self.pool2(x), hw, True, skip=acc)
        acc = ops.interpolate(self.pool3(x), hw, True, skip=acc)
        return self.conv(acc)


class FLD(nn.Module):
    """Flexible lightweight decoder: two UAFM fusions, widening 32->64->128 (stdc1)."""

    def __init__(self, encoder_channels, decoder_channels, num_class, fusion_type, act_type):
        super().__init__()
        d = decoder_channels
        self.stage6 = ConvBNAct(d[0], d[0])
        self.fusion1 = UAFM(encoder_channels[3], d[0], fusion_type)
        self.stage7 = ConvBNAct(d[0], d[1])
        self.fusion2 = UAFM(encoder_channels[2], d[1], fusion_type)
        self.stage8 = ConvBNAct(d[1], d[2])
        self.seg_head = ConvBNAct(d[2], num_class, 3, act_type=act_type)

    def forward(self, x3, x4, x5, size):
        x = self.stage7(self.fusion1(self.stage6(x5), x4))
        x = self.seg_head(self.stage8(self.fusion2(x, x3)))
        return ops.final_upsample(x, size, True)


class UAFM(nn.Module):
    """Unified attention fusion: alpha * up(x_high) + (1 - alpha) * conv(x_low)."""

    def __init__(self, in_channels, out_channels, fusion_type):
        super().__init__()
        hub = {"spatial": SpatialAttentionModule, "channel": ChannelAttentionModule}
        if fusion_type not in hub:
            raise ValueError(f"Unsupport fusion type: {fusion_type}.\n")
        self.conv = conv1x1(in_channels, out_channels)
        self.attention = hub[fusion_type](out_channels)

    def forward(self, x_high, x_low):
        x_low = self.conv(x_low)
        x_up = ops.interpolate(x_high, x_low.shape[2:], True)
        alpha = self.attention(x_up, x_low)
        return ops.gate(x_up, alpha, x_low, mode="blend")  # x_low + alpha * (x_up - x_low)


class SpatialAttentionModule(nn.Module):
    def __init__(self, out_channels):
        super().__init__()
        self.conv = conv1x1(4, 1)

    def forward(self, x_up, x_low):
        stats = [x_up.mean(1, keepdim=True), x_up.amax(1, keepdim=True),
                 x_low.mean(1, keepdim=True), x_low.amax(1, keepdim=True)]
        return torch.sigmoid(self.conv(torch.cat(stats, dim=1)))


class ChannelAttentionModule(nn.Module):
    def __init__(self, out_channels):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.max_pool = nn.AdaptiveMaxPool2d(1)
        self.conv = conv1x1(4 * out_channels, out_channels)

    def forward(self, x_up, x_low):
        stats = [self.avg_pool(x_up), self.max_pool(x_up), self.avg_pool(x_low), self.max_pool(x_low)]
        return torch.sigmoid(self.conv(torch.cat(stats, dim=1)))
