"""DeepLabV3 / DeepLabV3+ (SMP layout): ASPP with plain or depth-wise separable atrous branches.

Behavioural target: SMP ``DeepLabV3`` (encoder output stride 8, head x8) and
``DeepLabV3Plus`` (output stride 16, x4 decoder upsample + 48-channel
low-level projection, head x4) as used by reference models/__init__.py:42-44
and its KD teacher (``teacher_decoder='deeplabv3p'``, ResNet-101).  The
image-pooling branch is evaluated on the pooled vector and broadcast (a
bilinear resize of a 1x1 map is a broadcast), and every conv+BN+ReLU tail is
the fused HIP kernel.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ... import ops
from .base import ConvBNReLUSeq, SegmentationHead, SegmentationModel
from .encoders import get_encoder


class SeparableConv2d(nn.Sequential):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, bias=True):
        super().__init__(
            nn.Conv2d(in_channels, in_channels, kernel_size, stride=stride, padding=padding, dilation=dilation,
                      groups=in_channels, bias=False),
            nn.Conv2d(in_channels, out_channels, kernel_size=1, bias=bias))


class ASPPConv(ConvBNReLUSeq):
    def __init__(self, in_channels, out_channels, dilation):
        super().__init__(nn.Conv2d(in_channels, out_channels, 3, padding=dilation, dilation=dilation, bias=False),
                         nn.BatchNorm2d(out_channels), nn.ReLU())


class ASPPSeparableConv(ConvBNReLUSeq):
    def __init__(self, in_channels, out_channels, dilation):
        super().__init__(SeparableConv2d(in_channels, out_channels, 3, padding=dilation, dilation=dilation,
                                         bias=False),
                         nn.BatchNorm2d(out_channels), nn.ReLU())


class ASPPPooling(nn.Sequential):
    def __init__(self, in_channels, out_channels):
        super().__init__(nn.AdaptiveAvgPool2d(1), nn.Conv2d(in_channels, out_channels, 1, bias=False),
                         nn.BatchNorm2d(out_channels), nn.ReLU())

    def forward(self, x):
        y = ops.bn_act(self[1](x.mean(dim=(2, 3), keepdim=True)), self[2], "relu")
        return y.expand(-1, -1, x.shape[2], x.shape[3])


class ASPP(nn.Module):
    def __init__(self, in_channels, out_channels, atrous_rates, separable=False):
        super().__init__()
        branch = ASPPSeparableConv if separable else ASPPConv
        self.convs = nn.ModuleList(
            [ConvBNReLUSeq(nn.Conv2d(in_channels, out_channels, 1, bias=False), nn.BatchNorm2d(out_channels),
                           nn.ReLU())]
            + [branch(in_channels, out_channels, r) for r in tuple(atrous_rates)]
            + [ASPPPooling(in_channels, out_channels)])
        self.project = ConvBNReLUSeq(nn.Conv2d(5 * out_channels, out_channels, 1, bias=False),
                                     nn.BatchNorm2d(out_channels), nn.ReLU(), nn.Dropout(0.5))

    def forward(self, x):
        feats = [conv(x) for conv in self.convs]
        feats[-1] = feats[-1].to(feats[0].dtype)
        y = torch.cat(feats, dim=1)
        return self.project(y)


class DeepLabV3Decoder(nn.Sequential):
    def __init__(self, in_channels, out_channels=256, atrous_rates=(12, 24, 36)):
        super().__init__(ASPP(in_channels, out_channels, atrous_rates),
                         nn.Conv2d(out_channels, out_channels, 3, padding=1, bias=False),
                         nn.BatchNorm2d(out_channels), nn.ReLU())
        self.out_channels = out_channels

    def forward(self, *features):
        return ops.bn_act(self[1](self[0](features[-1])), self[2], "relu")


class DeepLabV3PlusDecoder(nn.Module):
    def __init__(self, encoder_channels, out_channels=256, atrous_rates=(12, 24, 36), output_stride=16):
        super().__init__()
        if output_stride not in (8, 16):
            raise ValueError(f"Output stride should be 8 or 16, got {output_stride}.")
        self.out_channels = out_channels
        self.output_stride = output_stride
        # SMP: aspp = Sequential(ASPP, SeparableConv2d, BN, ReLU) -- same child indices
        self.aspp = _AsppHead(encoder_channels[-1], out_channels, atrous_rates)
        self.scale_factor = 2 if output_stride == 8 else 4
        self.up = nn.UpsamplingBilinear2d(scale_factor=self.scale_factor)
        hi_in, hi_out = encoder_channels[-4], 48
        self.block1 = ConvBNReLUSeq(nn.Conv2d(hi_in, hi_out, 1, bias=False), nn.BatchNorm2d(hi_out), nn.ReLU())
        self.block2 = ConvBNReLUSeq(SeparableConv2d(hi_out + out_channels, out_channels, 3, padding=1, bias=False),
                                    nn.BatchNorm2d(out_channels), nn.ReLU())

    def forward(self, *features):
        a = self.aspp(features[-1])
        hi = self.block1(features[-4])
        a = ops.interpolate(a, hi.shape[2:], True)
        return self.block2(torch.cat([a, hi.to(a.dtype)], dim=1))


class _AsppHead(nn.Sequential):
    """``Sequential(ASPP, SeparableConv2d, BN, ReLU)`` with the BN+ReLU tail fused."""

    def __init__(self, in_channels, out_channels, atrous_rates):
        super().__init__(ASPP(in_channels, out_channels, atrous_rates, separable=True),
                         SeparableConv2d(out_channels, out_channels, 3, padding=1, bias=False),
                         nn.BatchNorm2d(out_channels), nn.ReLU())

    def forward(self, x):
        return ops.bn_act(self[1](self[0](x)), self[2], "relu")


class DeepLabV3(SegmentationModel):
    def __init__(self, encoder_name="resnet34", encoder_depth=5, encoder_weights="imagenet", decoder_channels=256,
                 in_channels=3, classes=1, upsampling=8):
        super().__init__()
        self.encoder = get_encoder(encoder_name, in_channels, encoder_depth, encoder_weights, output_stride=8)
        self.decoder = DeepLabV3Decoder(self.encoder.out_channels[-1], decoder_channels)
        self.segmentation_head = SegmentationHead(decoder_channels, classes, kernel_size=1, upsampling=upsampling)
        self.initialize()


class DeepLabV3Plus(SegmentationModel):
    def __init__(self, encoder_name="resnet34", encoder_depth=5, encoder_weights="imagenet",
                 encoder_output_stride=16, decoder_channels=256, decoder_atrous_rates=(12, 24, 36), in_channels=3,
                 classes=1, upsampling=4):
        super().__init__()
        if encoder_output_stride not in (8, 16):
            raise ValueError(f"Encoder output stride should be 8 or 16, got {encoder_output_stride}")
        self.encoder = get_encoder(encoder_name, in_channels, encoder_depth, encoder_weights,
                                   output_stride=encoder_output_stride)
        self.decoder = DeepLabV3PlusDecoder(self.encoder.out_channels, decoder_channels, decoder_atrous_rates,
                                            encoder_output_stride)
        self.segmentation_head = SegmentationHead(decoder_channels, classes, kernel_size=1, upsampling=upsampling)
        self.initialize()
