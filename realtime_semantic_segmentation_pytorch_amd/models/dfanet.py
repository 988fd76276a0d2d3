"""DFANet (arXiv:1904.02216) -- deep feature aggregation with cascaded Xception backbones.

Parity target: reference models/dfanet.py (DFANet :15-60, Encoder :63-93,
Decoder :96-130, EncoderBlock :133-143, FCAttention :146-161, XceptionBlock
:164-193).  The decoder's resize-and-sum chains run as fused resize+add
kernels; the final x4 resize is the deferred model output.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .modules import Activation, ConvBNAct, DSConvBNAct, DWConvBNAct, SegHead, conv1x1

_BACKBONE_CHANNELS = {"XceptionA": (48, 96, 192), "XceptionB": (32, 64, 128)}


def _scaled(t, f):
    return (t.shape[2] * f, t.shape[3] * f)


class DFANet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, backbone_type="XceptionA", expansion=4,
                 repeat_times=(4, 6, 4), use_extra_backbone=True, act_type="relu"):
        super().__init__()
        if len(repeat_times) != 3:
            raise AssertionError
        if backbone_type not in _BACKBONE_CHANNELS:
            raise NotImplementedError()
        ch = list(_BACKBONE_CHANNELS[backbone_type])
        self.use_extra_backbone = use_extra_backbone
        self.conv1 = ConvBNAct(n_channel, 8, 3, 2, act_type=act_type)
        self.backbone1 = Encoder([8, ch[0], ch[1]], ch, expansion, repeat_times, act_type)
        if use_extra_backbone:
            rotated = ch[2:] + ch[:2]  # each stage also receives the previous backbone's features
            cin = [a + b for a, b in zip(ch, rotated)]
            self.backbone2 = Encoder(cin, ch, expansion, repeat_times, act_type)
            self.backbone3 = Encoder(cin, ch, expansion, repeat_times, act_type)
            self.decoder = Decoder(ch[0], ch[2], num_class, act_type)
        else:
            self.seg_head = SegHead(ch[2], num_class, act_type)

    def forward(self, x, is_training=False):
        fc1, e2, e3, e4 = self.backbone1(self.conv1(x))
        if not self.use_extra_backbone:
            y = self.seg_head(fc1)
            return ops.final_upsample(y, _scaled(y, 16), True)
        enc1 = e2
        fc2, e2, e3, e4 = self.backbone2(ops.interpolate(fc1, _scaled(fc1, 4), True), e2, e3, e4)
        enc2 = e2
        fc3, enc3, _, _ = self.backbone3(ops.interpolate(fc2, _scaled(fc2, 4), True), e2, e3, e4)
        return self.decoder(enc1, enc2, enc3, fc1, fc2, fc3)


class Encoder(nn.Module):
    def __init__(self, in_channels, channels, expansion, repeat_times, act_type):
        super().__init__()
        if len(in_channels) != 3:
            raise AssertionError
        for i, name in enumerate(("enc2", "enc3", "enc4")):
            setattr(self, name, EncoderBlock(in_channels[i], channels[i], expansion, repeat_times[i], act_type))
        self.fc_attention = FCAttention(channels[2], act_type)

    def forward(self, x, x_enc2=None, x_enc3=None, x_enc4=None):
        outs = []
        for blk, prev in ((self.enc2, x_enc2), (self.enc3, x_enc3), (self.enc4, x_enc4)):
            x = blk(x if prev is None else torch.cat([x, prev], dim=1))
            outs.append(x)
        return (self.fc_attention(x), *outs)


class Decoder(nn.Module):
    def __init__(self, enc_channels, fc_channels, num_class, act_type, hid_channels=48):
        super().__init__()
        for i in (1, 2, 3):
            setattr(self, f"enc_conv{i}", ConvBNAct(enc_channels, hid_channels, 3, act_type=act_type, inplace=True))
        self.conv_enc = conv1x1(hid_channels, num_class)
        for i in (1, 2, 3):
            setattr(self, f"fc_conv{i}", SegHead(fc_channels, num_class, act_type))

    def forward(self, enc_x1, enc_x2, enc_x3, fc_x1, fc_x2, fc_x3):
        e = self.enc_conv1(enc_x1)
        hw = e.shape[2:]
        e = ops.interpolate(self.enc_conv2(enc_x2), hw, True, skip=e)
        e = ops.interpolate(self.enc_conv3(enc_x3), hw, True, skip=e)
        y = self.conv_enc(e)
        for head, f in ((self.fc_conv1, fc_x1), (self.fc_conv2, fc_x2), (self.fc_conv3, fc_x3)):
            y = ops.interpolate(head(f), hw, True, skip=y)
        return ops.final_upsample(y, _scaled(y, 4), True)


class EncoderBlock(nn.Module):
    def __init__(self, in_channels, out_channels, expansion, repeat_times, act_type):
        super().__init__()
        layers = [XceptionBlock(in_channels, out_channels, 2, expansion, act_type)]
        layers += [XceptionBlock(out_channels, out_channels, 1, expansion, act_type) for _ in range(repeat_times - 1)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return self.conv(x)


class FCAttention(nn.Module):
    """Global max-pool -> FC(1000) -> 1x1 ConvBNAct -> channel reweighting."""

    def __init__(self, channels, act_type, linear_channels=1000):
        super().__init__()
        self.channels = channels
        self.pool = nn.AdaptiveMaxPool2d(1)
        self.linear = nn.Linear(channels, linear_channels)
        self.conv = ConvBNAct(linear_channels, channels, 1, act_type=act_type, inplace=True)

    def forward(self, x):
        a = self.linear(self.pool(x).flatten(1))
        return x * self.conv(a[:, :, None, None])


class XceptionBlock(nn.Module):
    def __init__(self, in_channels, out_channels, stride, expansion, act_type):
        super().__init__()
        self.use_skip = in_channels == out_channels and stride == 1
        self.stride = stride
        hid = out_channels // expansion
        self.conv = nn.Sequential(
            DSConvBNAct(in_channels, hid, 3, act_type=act_type),
            DSConvBNAct(hid, hid, 3, act_type=act_type),
            DWConvBNAct(hid, out_channels, 3, stride, act_type=act_type, inplace=True),
            conv1x1(out_channels, out_channels),
            Activation(act_type))
        if stride > 1:
            self.conv_stride = conv1x1(in_channels, out_channels, 2)

    def forward(self, x):
        y = self.conv(x)
        if self.stride > 1:
            y = y + self.conv_stride(x)
        if self.use_skip:
            y = y + x
        return y
