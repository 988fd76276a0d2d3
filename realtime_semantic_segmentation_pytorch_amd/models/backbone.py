"""Native ResNet / MobileNetV2 backbones (torchvision is not available here).

Parity: reference models/backbone.py:4-57 wraps torchvision's ImageNet models
and returns 4 feature maps (strides 4, 8, 16, 32).  These re-implementations
use torchvision's exact attribute names (``conv1``, ``bn1``, ``layer1.0.conv1``,
``layer1.0.downsample.0`` ..., MobileNetV2 ``features`` indices), so
torchvision / SMP checkpoints load unchanged.  The convolution-BN-ReLU(+residual)
tails execute through the fused HIP ``bn_act`` kernel on GPU.

Pretrained weights: the reference downloads ImageNet weights at construction;
without network access ``pretrained=True`` looks for a torchvision-format
state dict at ``$RTSEG_PRETRAINED_DIR/<name>.pth`` and otherwise keeps the
random (torchvision-style) initialisation, with a warning.
"""
from __future__ import annotations

import os
import warnings

import torch
import torch.nn as nn

from .. import ops

RESNET_SPECS = {
    # name: (block, layers)
    "resnet18": ("basic", (2, 2, 2, 2)),
    "resnet34": ("basic", (3, 4, 6, 3)),
    "resnet50": ("bottleneck", (3, 4, 6, 3)),
    "resnet101": ("bottleneck", (3, 4, 23, 3)),
    "resnet152": ("bottleneck", (3, 8, 36, 3)),
    # ResNeXt (SMP / torchvision names): grouped 3x3 in every bottleneck, (groups, width per group)
    "resnext50_32x4d": ("bottleneck", (3, 4, 6, 3), 32, 4),
    "resnext101_32x4d": ("bottleneck", (3, 4, 23, 3), 32, 4),
    "resnext101_32x8d": ("bottleneck", (3, 4, 23, 3), 32, 8),
    "resnext101_32x16d": ("bottleneck", (3, 4, 23, 3), 32, 16),
    "resnext101_32x32d": ("bottleneck", (3, 4, 23, 3), 32, 32),
    "resnext101_32x48d": ("bottleneck", (3, 4, 23, 3), 32, 48),
}


def load_pretrained(module: nn.Module, name: str, strict: bool = False) -> bool:
    root = os.environ.get("RTSEG_PRETRAINED_DIR")
    path = os.path.join(root, f"{name}.pth") if root else None
    if path and os.path.isfile(path):
        sd = torch.load(path, map_location="cpu", weights_only=True)
        sd = sd.get("state_dict", sd) if isinstance(sd, dict) else sd
        own = module.state_dict()
        bad = [f"{k}: checkpoint {tuple(v.shape)} vs model {tuple(own[k].shape)}"
               for k, v in sd.items() if k in own and tuple(own[k].shape) != tuple(v.shape)]
        if bad:
            raise RuntimeError(f"pretrained weights {path} do not fit {name}: " + "; ".join(bad[:8]))
        missing, unexpected = module.load_state_dict(sd, strict=strict)
        if missing or unexpected:  # e.g. a classifier head the backbone wrapper drops
            warnings.warn(f"pretrained {name} ({path}): {len(missing)} missing key(s) {list(missing)[:6]}, "
                          f"{len(unexpected)} unexpected key(s) {list(unexpected)[:6]}")
        return True
    warnings.warn(f"pretrained weights for {name} not found (set RTSEG_PRETRAINED_DIR); "
                  "using random initialisation")
    return False


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, dilation, dilation=dilation, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, dilation, dilation=dilation, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = ops.conv_bn_act(x, self.conv1, self.bn1, "relu")
        return ops.conv_bn_act(out, self.conv2, self.bn2, "relu", residual=identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1, groups=1, base_width=64):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups  # torchvision's ResNeXt width rule
        self.conv1 = nn.Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, dilation, dilation=dilation, groups=groups, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = ops.conv_bn_act(x, self.conv1, self.bn1, "relu")
        out = ops.conv_bn_act(out, self.conv2, self.bn2, "relu")
        return ops.conv_bn_act(out, self.conv3, self.bn3, "relu", residual=identity)


class _ConvBN(nn.Sequential):
    """``downsample`` projection: keys ``.0.weight`` / ``.1.*`` (torchvision layout)."""

    def forward(self, x):
        return ops.conv_bn_act(x, self[0], self[1], "none")


class ResNet(nn.Module):
    """ResNet trunk returning (x4, x8, x16, x32) features.

    ``replace_stride_with_dilation`` = torchvision semantics (used by ICNet's
    dilated ResNet and DeepLab output-stride 8/16).
    """

    def __init__(self, resnet_type="resnet18", pretrained=False, replace_stride_with_dilation=(False, False, False),
                 in_channels=3):
        super().__init__()
        if resnet_type not in RESNET_SPECS:
            raise ValueError(f"Unsupported ResNet type: {resnet_type}.\n")
        kind, layers, *gw = RESNET_SPECS[resnet_type]
        self._groups, self._base_width = gw if gw else (1, 64)
        block = BasicBlock if kind == "basic" else Bottleneck
        self.resnet_type = resnet_type
        self.inplanes, self.dilation = 64, 1
        self.conv1 = nn.Conv2d(in_channels, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], 2, replace_stride_with_dilation[0])
        self.layer3 = self._make_layer(block, 256, layers[2], 2, replace_stride_with_dilation[1])
        self.layer4 = self._make_layer(block, 512, layers[3], 2, replace_stride_with_dilation[2])
        self.out_channels = [64 * block.expansion, 128 * block.expansion, 256 * block.expansion,
                             512 * block.expansion]
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if pretrained:
            load_pretrained(self, resnet_type)

    def _make_layer(self, block, planes, blocks, stride=1, dilate=False):
        downsample = None
        prev_dil = self.dilation
        if dilate:
            self.dilation *= stride
            stride = 1
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = _ConvBN(nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                                 nn.BatchNorm2d(planes * block.expansion))
        kw = {} if block is BasicBlock else {"groups": self._groups, "base_width": self._base_width}
        layers = [block(self.inplanes, planes, stride, downsample, prev_dil, **kw)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes, dilation=self.dilation, **kw) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def stem(self, x):
        return self.maxpool(ops.conv_bn_act(x, self.conv1, self.bn1, "relu"))

    def forward(self, x):
        x1 = self.layer1(self.stem(x))
        x2 = self.layer2(x1)
        x3 = self.layer3(x2)
        x4 = self.layer4(x3)
        return x1, x2, x3, x4


# ----------------------------------------------------------------- MobileNetV2
class ConvBNReLU6(nn.Sequential):
    """torchvision ``Conv2dNormActivation`` (keys ``.0`` conv, ``.1`` bn)."""

    def __init__(self, cin, cout, k=3, stride=1, groups=1):
        super().__init__(nn.Conv2d(cin, cout, k, stride, (k - 1) // 2, groups=groups, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU6(inplace=True))

    def forward(self, x):
        return ops.conv_bn_act(x, self[0], self[1], "relu6")


class InvertedResidual(nn.Module):
    def __init__(self, cin, cout, stride, expand_ratio):
        super().__init__()
        hid = int(round(cin * expand_ratio))
        self.use_res_connect = stride == 1 and cin == cout
        layers = []
        if expand_ratio != 1:
            layers.append(ConvBNReLU6(cin, hid, 1))
        layers += [ConvBNReLU6(hid, hid, 3, stride, groups=hid), nn.Conv2d(hid, cout, 1, bias=False),
                   nn.BatchNorm2d(cout)]
        self.conv = nn.Sequential(*layers)
        self.out_channels = cout

    def forward(self, x):
        h = x
        for layer in list(self.conv)[:-2]:
            h = layer(h)
        h = self.conv[-2](h)
        return ops.bn_act(h, self.conv[-1], "none", residual=x if self.use_res_connect else None)


def mobilenet_v2_features(width_mult=1.0):
    cfg = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1),
           (6, 160, 3, 2), (6, 320, 1, 1)]
    cin = int(32 * width_mult)
    feats = [ConvBNReLU6(3, cin, 3, 2)]
    for t, c, n, s in cfg:
        cout = int(c * width_mult)
        for i in range(n):
            feats.append(InvertedResidual(cin, cout, s if i == 0 else 1, t))
            cin = cout
    feats.append(ConvBNReLU6(cin, int(1280 * max(1.0, width_mult)), 1))
    return nn.Sequential(*feats)


class Mobilenetv2(nn.Module):
    """torchvision MobileNetV2 features split into 4 stages (x4, x8, x16, x32)."""

    def __init__(self, pretrained=False):
        super().__init__()
        f = mobilenet_v2_features()
        for m in f.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if pretrained:
            holder = nn.Module()
            holder.features = f
            load_pretrained(holder, "mobilenet_v2")
        self.layer1 = f[:4]
        self.layer2 = f[4:7]
        self.layer3 = f[7:14]
        self.layer4 = f[14:18]
        self.out_channels = [24, 32, 96, 320]

    def forward(self, x):
        x1 = self.layer1(x)
        x2 = self.layer2(x1)
        x3 = self.layer3(x2)
        x4 = self.layer4(x3)
        return x1, x2, x3, x4
