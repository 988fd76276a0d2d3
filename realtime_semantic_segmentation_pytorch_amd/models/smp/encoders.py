"""SMP-style encoders: ResNet-18/34/50/101/152, ResNeXt-50/101 (32xNd), MobileNetV2, the
Mix Transformers MiT-B0..B5 (``mit.py``) and VGG / DenseNet / EfficientNet-B0..B7 / SE-ResNet /
SE-ResNeXt (``encoders_extra.py``).

Behavioural target: SMP's ``ResNetEncoder`` / ``MobileNetV2Encoder`` (the
torchvision networks with the classifier removed; ``forward`` returns the
``depth + 1`` stage outputs [x, /2, /4, /8, /16, /32]; ``make_dilated``
replaces the strides of the last one or two stages by dilation 2 / 4 in
*every* conv of the stage -- SMP's rule, which differs from torchvision's
``replace_stride_with_dilation``).  Built on the native backbones of
:mod:`..backbone`, whose BN(+residual)+ReLU tails run on the fused HIP kernel.
"""
from __future__ import annotations

import torch.nn as nn

from ... import ops
from ..backbone import RESNET_SPECS, ResNet, load_pretrained, mobilenet_v2_features
from .mit import MIT_SPECS, MixVisionTransformerEncoder

_RESNET_CHANNELS = {"basic": (3, 64, 64, 128, 256, 512), "bottleneck": (3, 64, 256, 512, 1024, 2048)}


def replace_strides_with_dilation(module: nn.Module, dilation_rate: int):
    for m in module.modules():
        if isinstance(m, nn.Conv2d):
            m.stride = (1, 1)
            m.dilation = (dilation_rate, dilation_rate)
            kh, kw = m.kernel_size
            m.padding = ((kh // 2) * dilation_rate, (kw // 2) * dilation_rate)


class _EncoderMixin:
    """``out_channels`` / ``output_stride`` bookkeeping and SMP's ``make_dilated``."""

    _output_stride = 32

    def _set_channels(self, channels, depth):
        self._depth = depth
        self._out_channels = tuple(channels)
        self.out_channels = self._out_channels[: depth + 1]

    @property
    def output_stride(self):
        return min(self._output_stride, 2 ** self._depth)

    def make_dilated(self, output_stride):
        if output_stride == 32:
            return
        if output_stride == 16:
            plan = ((5, 2),)
        elif output_stride == 8:
            plan = ((4, 2), (5, 4))
        else:
            raise ValueError(f"Output stride should be 16 or 8, got {output_stride}.")
        self._output_stride = output_stride
        stages = self.get_stages()
        for idx, rate in plan:
            replace_strides_with_dilation(stages[idx], rate)

    def forward(self, x):
        feats = [x]
        for stage in self._stage_fns()[: self._depth]:
            x = stage(x)
            feats.append(x)
        return feats


class ResNetEncoder(_EncoderMixin, ResNet):
    def __init__(self, name, depth=5):
        super().__init__(name)
        self._set_channels(_RESNET_CHANNELS[RESNET_SPECS[name][0]], depth)

    def get_stages(self):
        return [nn.Identity(), nn.ModuleList([self.conv1, self.bn1]), nn.ModuleList([self.maxpool, self.layer1]),
                self.layer2, self.layer3, self.layer4]

    def _stage_fns(self):
        return [lambda x: ops.conv_bn_act(x, self.conv1, self.bn1, "relu"),
                lambda x: self.layer1(self.maxpool(x)), self.layer2, self.layer3, self.layer4]


class MobileNetV2Encoder(_EncoderMixin, nn.Module):
    def __init__(self, depth=5):
        super().__init__()
        self.features = mobilenet_v2_features()
        self._set_channels((3, 16, 24, 32, 96, 1280), depth)

    def get_stages(self):
        f = self.features
        return [nn.Identity(), f[:2], f[2:4], f[4:7], f[7:14], f[14:]]

    def _stage_fns(self):
        return self.get_stages()[1:]


def _extra():
    from . import encoders_extra

    return encoders_extra


ENCODERS = tuple(RESNET_SPECS) + ("mobilenet_v2",) + tuple(MIT_SPECS) + (
    "vgg11", "vgg11_bn", "vgg13", "vgg13_bn", "vgg16", "vgg16_bn", "vgg19", "vgg19_bn",
    "densenet121", "densenet161", "densenet169", "densenet201",
    "efficientnet-b0", "efficientnet-b1", "efficientnet-b2", "efficientnet-b3",
    "efficientnet-b4", "efficientnet-b5", "efficientnet-b6", "efficientnet-b7",
    "se_resnet50", "se_resnet101", "se_resnet152", "se_resnext50_32x4d", "se_resnext101_32x4d")


def get_encoder(name, in_channels=3, depth=5, weights=None, output_stride=32):
    if name is None:
        raise ValueError("config.encoder must be set for model='smp'")
    if name in MIT_SPECS:
        # SMP's MixVisionTransformerEncoder: 3 input channels only, no dilated mode
        if in_channels != 3:
            raise ValueError("MixVisionTransformer encoder does not support in_channels setting other than 3")
        enc = MixVisionTransformerEncoder(name, depth)
        if weights is not None:
            load_pretrained(enc, name)
        enc.make_dilated(output_stride)
        return enc
    if name in RESNET_SPECS:
        enc = ResNetEncoder(name, depth)
    elif name == "mobilenet_v2":
        enc = MobileNetV2Encoder(depth)
    elif name in ENCODERS:
        enc = _extra().build_extra_encoder(name, depth)
    else:
        raise ValueError(f"Unsupported encoder `{name}`; available: {', '.join(ENCODERS)}")
    if weights is not None:
        # SMP downloads ImageNet weights; offline, a torchvision-format file is looked up instead
        load_pretrained(enc, name)
    if in_channels != 3:
        _patch_first_conv(enc, in_channels)
    enc.make_dilated(output_stride)
    return enc


def _patch_first_conv(enc, in_channels):
    import torch
    for m in enc.modules():
        if isinstance(m, nn.Conv2d) and m.in_channels == 3:
            w = m.weight.detach()
            m.in_channels = in_channels
            if in_channels == 1:
                nw = w.sum(1, keepdim=True)
            else:
                reps = -(-in_channels // 3)
                nw = torch.cat([w] * reps, dim=1)[:, :in_channels] * (3.0 / in_channels)
            m.weight = nn.Parameter(nw)
            return
