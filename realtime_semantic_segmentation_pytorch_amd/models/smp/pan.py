"""PAN decoder (SMP layout): feature pyramid attention + global attention upsample blocks.

Behavioural target: SMP ``PAN`` (reference models/__init__.py:42-44, 67-71):
encoder output stride 16 by default, FPA on the deepest feature, three GAU
blocks up to 1/4, 3x3 head with x4 upsampling.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ... import ops
from .base import SegmentationHead, SegmentationModel
from .encoders import get_encoder


class ConvBnRelu(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1, bias=True,
                 add_relu=True, interpolate=False):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias)
        self.add_relu = add_relu
        self.interpolate = interpolate
        self.bn = nn.BatchNorm2d(out_channels)
        self.activation = nn.ReLU(inplace=True)

    def forward(self, x):
        y = ops.conv_bn_act(x, self.conv, self.bn, "relu" if self.add_relu else "none")
        if self.interpolate:
            y = ops.interpolate(y, (y.shape[2] * 2, y.shape[3] * 2), True)
        return y


class FPABlock(nn.Module):
    def __init__(self, in_channels, out_channels, upscale_mode="bilinear"):
        super().__init__()
        if upscale_mode != "bilinear":
            raise NotImplementedError("only bilinear upscaling is supported")
        self.upscale_mode = upscale_mode
        self.align_corners = True
        self.branch1 = nn.Sequential(nn.AdaptiveAvgPool2d(1), ConvBnRelu(in_channels, out_channels, 1))
        self.mid = nn.Sequential(ConvBnRelu(in_channels, out_channels, 1))
        self.down1 = nn.Sequential(nn.MaxPool2d(2, 2), ConvBnRelu(in_channels, 1, 7, padding=3))
        self.down2 = nn.Sequential(nn.MaxPool2d(2, 2), ConvBnRelu(1, 1, 5, padding=2))
        self.down3 = nn.Sequential(nn.MaxPool2d(2, 2), ConvBnRelu(1, 1, 3, padding=1), ConvBnRelu(1, 1, 3, padding=1))
        self.conv2 = ConvBnRelu(1, 1, 5, padding=2)
        self.conv1 = ConvBnRelu(1, 1, 7, padding=3)

    def forward(self, x):
        h, w = x.shape[2:]
        b1 = self.branch1(x)  # [N, C, 1, 1]: its bilinear resize is a broadcast
        mid = self.mid(x)
        x1 = self.down1(x)
        x2 = self.down2(x1)
        x3 = self.down3(x2)
        y = ops.interpolate(x3, (h // 4, w // 4), True, skip=self.conv2(x2))
        y = ops.interpolate(y, (h // 2, w // 2), True, skip=self.conv1(x1))
        y = ops.interpolate(y, (h, w), True)
        return y * mid + b1


class GAUBlock(nn.Module):
    def __init__(self, in_channels, out_channels, upscale_mode="bilinear"):
        super().__init__()
        if upscale_mode != "bilinear":
            raise NotImplementedError("only bilinear upscaling is supported")
        self.upscale_mode = upscale_mode
        self.align_corners = True
        self.conv1 = nn.Sequential(nn.AdaptiveAvgPool2d(1), ConvBnRelu(out_channels, out_channels, 1, add_relu=False),
                                   nn.Sigmoid())
        self.conv2 = ConvBnRelu(in_channels, out_channels, 3, padding=1)

    def forward(self, x, y):
        """x: low-level feature, y: high-level feature."""
        z = self.conv2(x) * self.conv1(y)
        return ops.interpolate(y, x.shape[2:], True, skip=z.to(y.dtype))


class PANDecoder(nn.Module):
    def __init__(self, encoder_channels, decoder_channels, upscale_mode="bilinear"):
        super().__init__()
        self.fpa = FPABlock(encoder_channels[-1], decoder_channels)
        self.gau3 = GAUBlock(encoder_channels[-2], decoder_channels, upscale_mode)
        self.gau2 = GAUBlock(encoder_channels[-3], decoder_channels, upscale_mode)
        self.gau1 = GAUBlock(encoder_channels[-4], decoder_channels, upscale_mode)

    def forward(self, *features):
        x5 = self.fpa(features[-1])
        x4 = self.gau3(features[-2], x5)
        x3 = self.gau2(features[-3], x4)
        return self.gau1(features[-4], x3)


class PAN(SegmentationModel):
    def __init__(self, encoder_name="resnet34", encoder_weights="imagenet", encoder_output_stride=16,
                 decoder_channels=32, in_channels=3, classes=1, upsampling=4):
        super().__init__()
        if encoder_output_stride not in (8, 16, 32):
            raise ValueError(f"PAN support output stride 8, 16 and 32, got {encoder_output_stride}.")
        self.encoder = get_encoder(encoder_name, in_channels, 5, encoder_weights, output_stride=encoder_output_stride)
        self.decoder = PANDecoder(self.encoder.out_channels, decoder_channels)
        self.segmentation_head = SegmentationHead(decoder_channels, classes, kernel_size=3, upsampling=upsampling)
        self.initialize()
