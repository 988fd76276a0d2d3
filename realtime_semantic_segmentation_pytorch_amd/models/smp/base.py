"""Shared SMP-compatible pieces: model base, segmentation head, Conv2dReLU, init.

Behavioural target: segmentation_models_pytorch (the reference's
``models/__init__.py:42-44,67-81`` bridge; SMP itself is not installed here, so
module trees follow the SMP 0.3 layout -- ``encoder.*``, ``decoder.*``,
``segmentation_head.0.*`` -- and checkpoint interchange with real SMP
checkpoints is "parity unpinned").  Execution differs from SMP: decoder
conv+BN+ReLU tails run through the fused HIP ``bn_act`` kernel, and the head's
final bilinear upsample is a deferrable model output (``ops.final_upsample``)
that the fused loss consumes directly in training.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ... import ops


class Conv2dReLU(nn.Sequential):
    """conv (bias iff no BN) -> BN | Identity -> ReLU; children ``0 / 1 / 2``."""

    def __init__(self, in_channels, out_channels, kernel_size, padding=0, stride=1, use_batchnorm=True):
        conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                         bias=not use_batchnorm)
        bn = nn.BatchNorm2d(out_channels) if use_batchnorm else nn.Identity()
        super().__init__(conv, bn, nn.ReLU(inplace=True))

    def forward(self, x):
        y = self[0](x)
        if isinstance(self[1], nn.BatchNorm2d):
            return ops.bn_act(y, self[1], "relu")
        return torch.relu(y)


class ConvBNReLUSeq(nn.Sequential):
    """Generic ``Sequential(conv-like, BatchNorm2d, ReLU[, extra...])`` with a fused tail."""

    def forward(self, x):
        y = ops.conv_bn_act(x, self[0], self[1], "relu")
        for m in list(self)[3:]:
            y = m(y)
        return y


class SegmentationHead(nn.Sequential):
    """conv(k) -> bilinear x``upsampling`` (align_corners=True) -> identity activation."""

    def __init__(self, in_channels, out_channels, kernel_size=3, upsampling=1):
        conv = nn.Conv2d(in_channels, out_channels, kernel_size, padding=kernel_size // 2)
        up = nn.UpsamplingBilinear2d(scale_factor=upsampling) if upsampling > 1 else nn.Identity()
        super().__init__(conv, up, nn.Identity())
        self.upsampling = upsampling

    def forward(self, x):
        y = self[0](x)
        if self.upsampling > 1:
            return ops.final_upsample(y, (y.shape[2] * self.upsampling, y.shape[3] * self.upsampling), True)
        return y


def initialize_decoder(module: nn.Module):
    for m in module.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_uniform_(m.weight, mode="fan_in", nonlinearity="relu")
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.Linear):
            nn.init.xavier_uniform_(m.weight)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)


def initialize_head(module: nn.Module):
    for m in module.modules():
        if isinstance(m, (nn.Linear, nn.Conv2d)):
            nn.init.xavier_uniform_(m.weight)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)


class SegmentationModel(nn.Module):
    """encoder -> decoder(*features) -> segmentation_head."""

    def initialize(self):
        initialize_decoder(self.decoder)
        initialize_head(self.segmentation_head)

    def check_input_shape(self, x):
        h, w = x.shape[-2:]
        s = self.encoder.output_stride
        if h % s or w % s:
            raise RuntimeError(f"Wrong input shape height={h}, width={w}. Expected image height and width "
                               f"divisible by {s}.")

    def forward(self, x, is_training=False):
        self.check_input_shape(x)
        features = self.encoder(x)
        return self.segmentation_head(self.decoder(*features))

    @torch.no_grad()
    def predict(self, x):
        if self.training:
            self.eval()
        return self.forward(x)
