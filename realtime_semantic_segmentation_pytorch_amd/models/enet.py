"""ENet (arXiv:1606.02147).

Parity target: reference models/enet.py (ENet :14-35, InitialBlock :38-48,
BottleNeck1/23/45 :51-116, Bottleneck :119-184 with regular / downsampling
(max-pool indices) / upsampling (max-unpool) / dilated / asymmetric variants,
Upsample :187-205).  Module names match the reference (430 state_dict keys).
The final 1x1 + bilinear x2 (align_corners=False) is a deferred model output.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .modules import Activation, ConvBNAct, conv1x1

# the 8 bottlenecks of stages 2 and 3: (type, dilation)
_STAGE23 = (("regular", 1), ("dilate", 2), ("asymmetric", 1), ("dilate", 4), ("regular", 1),
            ("dilate", 8), ("asymmetric", 1), ("dilate", 16))


class ENet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="prelu", upsample_type="deconvolution"):
        super().__init__()
        self.initial = InitialBlock(n_channel, 16, act_type)
        self.bottleneck1 = BottleNeck1(16, 64, act_type)
        self.bottleneck2 = BottleNeck23(64, 128, act_type, True)
        self.bottleneck3 = BottleNeck23(128, 128, act_type, False)
        self.bottleneck4 = BottleNeck45(128, 64, act_type, upsample_type, True)
        self.bottleneck5 = BottleNeck45(64, 16, act_type, upsample_type, False)
        self.fullconv = Upsample(16, num_class, scale_factor=2, act_type=act_type)

    def forward(self, x, is_training=False):
        x = self.initial(x)
        x, idx1 = self.bottleneck1(x)  # 1/4
        x, idx2 = self.bottleneck2(x)  # 1/8
        x = self.bottleneck3(x)
        x = self.bottleneck5(self.bottleneck4(x, idx2), idx1)
        return self.fullconv(x, final=True)


class InitialBlock(nn.Module):
    """conv (cout - cin channels, s2) || max-pool, concatenated."""

    def __init__(self, in_channels, out_channels, act_type, kernel_size=3, **kwargs):
        super().__init__()
        if out_channels <= in_channels:
            raise AssertionError("out_channels should be larger than in_channels.\n")
        self.conv = ConvBNAct(in_channels, out_channels - in_channels, kernel_size, 2, act_type=act_type, **kwargs)
        self.pool = nn.MaxPool2d(3, 2, 1)
        self.widths = (out_channels - in_channels, in_channels)

    def forward(self, x):
        # K11: the conv branch's BN kernel stores into its slice of one concat buffer and the max
        # pool runs inside the cat node into the other (ops.ConcatSink, as BiSeNetV2's stem); with
        # unaligned widths (ENet's 13 || 3) or an unfused activation the parts are copied in.
        # Under autocast the conv branch is bf16 while max-pooling the fp32 input image stays fp32:
        # a plain cat would promote the block -- and every activation of the 10 networks built on
        # it (ENet, ERFNet, LEDNet, AGLNet, ESNet, FDDWNet, ...) -- to fp32, with a bf16 cast before
        # each conv (profiles/r4_zoo_models).  Max pooling commutes with the rounding, so the cast
        # of the pooled branch is exact w.r.t. pooling the rounded input
        sink = ops.ConcatSink(self.widths)
        y = self.conv(x, sink=(sink, 0))
        pl = self.pool
        return sink.cat([y, sink.max_pool(1, x, pl.kernel_size, pl.stride, pl.padding, dtype=y.dtype)])


class BottleNeck1(nn.Module):
    def __init__(self, in_channels, out_channels, act_type="prelu", drop_p=0.01):
        super().__init__()
        self.conv_pool = Bottleneck(in_channels, out_channels, "downsampling", act_type, drop_p=drop_p)
        self.conv_regular = nn.Sequential(
            *[Bottleneck(out_channels, out_channels, "regular", act_type, drop_p=drop_p) for _ in range(4)])

    def forward(self, x):
        x, idx = self.conv_pool(x)
        return self.conv_regular(x), idx


class BottleNeck23(nn.Module):
    def __init__(self, in_channels, out_channels, act_type="prelu", downsample=True):
        super().__init__()
        self.downsample = downsample
        if downsample:
            self.conv_pool = Bottleneck(in_channels, out_channels, "downsampling", act_type=act_type)
        self.conv_regular = nn.Sequential(
            *[Bottleneck(out_channels, out_channels, t, act_type, dilation=d) for t, d in _STAGE23])

    def forward(self, x):
        if not self.downsample:
            return self.conv_regular(x)
        x, idx = self.conv_pool(x)
        return self.conv_regular(x), idx


class BottleNeck45(nn.Module):
    def __init__(self, in_channels, out_channels, act_type="prelu", upsample_type=None, extra_conv=False):
        super().__init__()
        self.extra_conv = extra_conv
        self.conv_unpool = Bottleneck(in_channels, out_channels, "upsampling", act_type, upsample_type)
        self.conv_regular = Bottleneck(out_channels, out_channels, "regular", act_type)
        if extra_conv:
            self.conv_extra = Bottleneck(out_channels, out_channels, "regular", act_type)

    def forward(self, x, indices):
        x = self.conv_regular(self.conv_unpool(x, indices))
        return self.conv_extra(x) if self.extra_conv else x


class Bottleneck(nn.Module):
    """ENet bottleneck: 1x1 reduce (x0.25) -> main conv -> 1x1 expand + dropout, with a
    type-specific shortcut (identity, max-pool + 1x1, or 1x1 + max-unpool)."""

    def __init__(self, in_channels, out_channels, conv_type, act_type="prelu", upsample_type="regular",
                 dilation=1, drop_p=0.1, shrink_ratio=0.25):
        super().__init__()
        self.conv_type = conv_type
        hid = int(in_channels * shrink_ratio)
        if conv_type == "regular":
            main = [ConvBNAct(in_channels, hid, 1), ConvBNAct(hid, hid)]
        elif conv_type == "downsampling":
            self.left_pool = nn.MaxPool2d(2, 2, return_indices=True)
            self.left_conv = ConvBNAct(in_channels, out_channels, 1)
            main = [ConvBNAct(in_channels, hid, 3, 2), ConvBNAct(hid, hid)]
        elif conv_type == "upsampling":
            self.left_conv = ConvBNAct(in_channels, out_channels, 1)
            self.left_pool = nn.MaxUnpool2d(2, 2)
            main = [ConvBNAct(in_channels, hid, 1),
                    Upsample(hid, hid, scale_factor=2, kernel_size=3, upsample_type=upsample_type)]
        elif conv_type == "dilate":
            main = [ConvBNAct(in_channels, hid, 1), ConvBNAct(hid, hid, dilation=dilation)]
        elif conv_type == "asymmetric":
            main = [ConvBNAct(in_channels, hid, 1), ConvBNAct(hid, hid, (5, 1)), ConvBNAct(hid, hid, (1, 5))]
        else:
            raise ValueError(f"[!] Unsupport convolution type: {conv_type}")
        self.right_init_conv = nn.Sequential(*main)
        self.right_last_conv = nn.Sequential(conv1x1(hid, out_channels), nn.Dropout(drop_p))
        self.act = Activation(act_type)

    def forward(self, x, indices=None):
        branch = self.right_last_conv(self.right_init_conv(x))
        if self.conv_type == "downsampling":
            pooled, indices = self.left_pool(x)
            return self.act(self.left_conv(pooled) + branch), indices
        if self.conv_type == "upsampling":
            if indices is None:
                raise ValueError("Upsampling-type conv needs pooling indices.")
            return self.act(self.left_pool(self.left_conv(x), indices) + branch)
        return self.act(x + branch)


class Upsample(nn.Module):
    """x`scale_factor`: transposed conv ('deconvolution') or 1x1 ConvBNAct + bilinear."""

    def __init__(self, in_channels, out_channels, scale_factor=2, kernel_size=None, upsample_type=None,
                 act_type="relu"):
        super().__init__()
        self.scale_factor = scale_factor
        self.deconv = upsample_type == "deconvolution"
        if self.deconv:
            k = 2 * scale_factor - 1 if kernel_size is None else kernel_size
            self.up_conv = nn.ConvTranspose2d(in_channels, out_channels, kernel_size=k, stride=scale_factor,
                                              padding=(k - 1) // 2, output_padding=1, bias=False)
        else:
            self.up_conv = nn.Sequential(ConvBNAct(in_channels, out_channels, 1, act_type=act_type),
                                         nn.Upsample(scale_factor=scale_factor, mode="bilinear"))

    def forward(self, x, final=False):
        if self.deconv:
            return self.up_conv(x)
        y = self.up_conv[0](x)
        size = (y.shape[2] * self.scale_factor, y.shape[3] * self.scale_factor)
        if final:
            return ops.final_upsample(y, size, align_corners=False)
        return ops.interpolate(y, size, align_corners=False)
