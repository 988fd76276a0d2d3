"""More SMP encoders: VGG-11/13/16/19 (+BN), DenseNet-121/161/169/201, EfficientNet-B0..B7 and
SE-ResNet-50/101/152 / SE-ResNeXt-50/101 (32x4d).

The reference forwards any ``config.encoder`` name to segmentation_models_pytorch
(reference models/__init__.py:67-81), which is not installed here; these are native
re-implementations with SMP's module trees -- the torchvision VGG / DenseNet layouts
(``features.*``), lukemelas' EfficientNet-PyTorch layout (``_conv_stem``, ``_blocks.N._expand_conv``,
...) and Cadene's pretrainedmodels SENet layout (``layer0.conv1``, ``layerN.M.se_module.fc1``) --
so checkpoints saved by an SMP model load by key.  Key-for-key parity against SMP itself is
unpinned (the library is not importable here); shapes, stage channels and strides follow the
published architectures and SMP's ``get_stages`` / ``out_channels`` tables.

Every encoder returns SMP's ``depth + 1`` features [x, /2, /4, /8, /16, /32] (VGG: its stage
outputs, the first at full resolution, as SMP's VGGEncoder does).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import ops
from .encoders import _EncoderMixin


# ----------------------------------------------------------------------------------------- VGG
_VGG_CFGS = {
    "A": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "B": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "D": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "E": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"],
}
VGG_SPECS = {"vgg11": ("A", False), "vgg11_bn": ("A", True), "vgg13": ("B", False), "vgg13_bn": ("B", True),
             "vgg16": ("D", False), "vgg16_bn": ("D", True), "vgg19": ("E", False), "vgg19_bn": ("E", True)}


class VGGEncoder(_EncoderMixin, nn.Module):
    """torchvision ``vgg*`` ``features`` (keys ``features.N.*``), classifier removed."""

    def __init__(self, name, depth=5):
        super().__init__()
        cfg, bn = VGG_SPECS[name]
        layers, cin = [], 3
        for v in _VGG_CFGS[cfg]:
            if v == "M":
                layers.append(nn.MaxPool2d(2, 2))
                continue
            layers.append(nn.Conv2d(cin, v, 3, padding=1))
            if bn:
                layers.append(nn.BatchNorm2d(v))
            layers.append(nn.ReLU(inplace=True))
            cin = v
        self.features = nn.Sequential(*layers)
        self._set_channels((64, 128, 256, 512, 512, 512), depth)

    def make_dilated(self, output_stride):
        if output_stride != 32:
            raise ValueError("'VGG' models do not support dilated mode due to Max Pooling operations "
                             "for downsampling!")

    def get_stages(self):
        stages, cur = [], []
        for m in self.features:
            if isinstance(m, nn.MaxPool2d):
                stages.append(nn.Sequential(*cur))
                cur = []
            cur.append(m)
        stages.append(nn.Sequential(*cur))
        return stages

    def forward(self, x):
        feats = []
        for stage in self.get_stages()[: self._depth + 1]:
            x = stage(x)
            feats.append(x)
        return feats


# ------------------------------------------------------------------------------------ DenseNet
DENSENET_SPECS = {"densenet121": (32, (6, 12, 24, 16), 64), "densenet161": (48, (6, 12, 36, 24), 96),
                  "densenet169": (32, (6, 12, 32, 32), 64), "densenet201": (32, (6, 12, 48, 32), 64)}


class _DenseLayer(nn.Module):
    def __init__(self, cin, growth, bn_size=4):
        super().__init__()
        self.norm1 = nn.BatchNorm2d(cin)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv1 = nn.Conv2d(cin, bn_size * growth, 1, bias=False)
        self.norm2 = nn.BatchNorm2d(bn_size * growth)
        self.relu2 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(bn_size * growth, growth, 3, padding=1, bias=False)

    def forward(self, feats):
        x = torch.cat(feats, 1) if isinstance(feats, (list, tuple)) else feats
        y = self.conv1(ops.bn_act(x, self.norm1, "relu"))
        return self.conv2(ops.bn_act(y, self.norm2, "relu"))


class _DenseBlock(nn.ModuleDict):
    def __init__(self, n, cin, growth):
        super().__init__()
        for i in range(n):
            self[f"denselayer{i + 1}"] = _DenseLayer(cin + i * growth, growth)

    def forward(self, x):
        feats = [x]
        for layer in self.values():
            feats.append(layer(feats))
        return torch.cat(feats, 1)


class _Transition(nn.Sequential):
    def __init__(self, cin, cout):
        super().__init__()
        self.add_module("norm", nn.BatchNorm2d(cin))
        self.add_module("relu", nn.ReLU(inplace=True))
        self.add_module("conv", nn.Conv2d(cin, cout, 1, bias=False))
        self.add_module("pool", nn.AvgPool2d(2, 2))


class _TransitionWithSkip(nn.Module):
    """SMP: the transition's post-ReLU activation is the stage's skip feature."""

    def __init__(self, module):
        super().__init__()
        self.module = module

    def forward(self, x):
        skip = ops.bn_act(x, self.module.norm, "relu")
        return self.module.pool(self.module.conv(skip)), skip


class DenseNetEncoder(_EncoderMixin, nn.Module):
    """torchvision ``densenet*`` (keys ``features.conv0``, ``features.denseblockN.denselayerM.*``,
    ``features.transitionN.*``, ``features.norm5``), classifier removed."""

    def __init__(self, name, depth=5):
        super().__init__()
        growth, blocks, init = DENSENET_SPECS[name]
        f = nn.Sequential()
        f.add_module("conv0", nn.Conv2d(3, init, 7, 2, 3, bias=False))
        f.add_module("norm0", nn.BatchNorm2d(init))
        f.add_module("relu0", nn.ReLU(inplace=True))
        f.add_module("pool0", nn.MaxPool2d(3, 2, 1))
        c, chans = init, [3, init]
        for i, n in enumerate(blocks):
            f.add_module(f"denseblock{i + 1}", _DenseBlock(n, c, growth))
            c += n * growth
            chans.append(c)
            if i != len(blocks) - 1:
                f.add_module(f"transition{i + 1}", _Transition(c, c // 2))
                c //= 2
        f.add_module("norm5", nn.BatchNorm2d(c))
        self.features = f
        chans[-1] = c
        self._set_channels(chans, depth)

    def make_dilated(self, output_stride):
        if output_stride != 32:
            raise ValueError("DenseNet encoders do not support dilated mode due to pooling operation for downsampling!")

    def get_stages(self):
        f = self.features
        return [nn.Identity(), nn.Sequential(f.conv0, f.norm0, f.relu0),
                nn.Sequential(f.pool0, f.denseblock1, _TransitionWithSkip(f.transition1)),
                nn.Sequential(f.denseblock2, _TransitionWithSkip(f.transition2)),
                nn.Sequential(f.denseblock3, _TransitionWithSkip(f.transition3)),
                nn.Sequential(f.denseblock4, f.norm5)]

    def forward(self, x):
        f = self.features
        stages = [lambda t: t,
                  lambda t: ops.conv_bn_act(t, f.conv0, f.norm0, "relu"),
                  lambda t: _TransitionWithSkip(f.transition1)(f.denseblock1(f.pool0(t))),
                  lambda t: _TransitionWithSkip(f.transition2)(f.denseblock2(t)),
                  lambda t: _TransitionWithSkip(f.transition3)(f.denseblock3(t)),
                  lambda t: f.norm5(f.denseblock4(t))]
        feats = []
        for stage in stages[: self._depth + 1]:
            x = stage(x)
            if isinstance(x, tuple):
                x, skip = x
                feats.append(skip)
            else:
                feats.append(x)
        return feats


# -------------------------------------------------------------------------------- EfficientNet
# (width, depth, resolution, dropout) -- EfficientNet-PyTorch's efficientnet_params()
EFFNET_PARAMS = {"efficientnet-b0": (1.0, 1.0, 224, 0.2), "efficientnet-b1": (1.0, 1.1, 240, 0.2),
                 "efficientnet-b2": (1.1, 1.2, 260, 0.3), "efficientnet-b3": (1.2, 1.4, 300, 0.3),
                 "efficientnet-b4": (1.4, 1.8, 380, 0.4), "efficientnet-b5": (1.6, 2.2, 456, 0.4),
                 "efficientnet-b6": (1.8, 2.6, 528, 0.5), "efficientnet-b7": (2.0, 3.1, 600, 0.5)}
# SMP's stage split (block indices) and out_channels per model
_EFFNET_SMP = {"efficientnet-b0": ((3, 5, 9, 16), (3, 32, 24, 40, 112, 320)),
               "efficientnet-b1": ((5, 8, 16, 23), (3, 32, 24, 40, 112, 320)),
               "efficientnet-b2": ((5, 8, 16, 23), (3, 32, 24, 48, 120, 352)),
               "efficientnet-b3": ((5, 8, 18, 26), (3, 40, 32, 48, 136, 384)),
               "efficientnet-b4": ((6, 10, 22, 32), (3, 48, 32, 56, 160, 448)),
               "efficientnet-b5": ((8, 13, 27, 39), (3, 48, 40, 64, 176, 512)),
               "efficientnet-b6": ((9, 15, 31, 45), (3, 56, 40, 72, 200, 576)),
               "efficientnet-b7": ((11, 18, 38, 55), (3, 64, 48, 80, 224, 640))}
# repeats, kernel, stride, expand, in, out (se ratio 0.25 everywhere)
_EFFNET_BLOCKS = ((1, 3, 1, 1, 32, 16), (2, 3, 2, 6, 16, 24), (2, 5, 2, 6, 24, 40), (3, 3, 2, 6, 40, 80),
                  (3, 5, 1, 6, 80, 112), (4, 5, 2, 6, 112, 192), (1, 3, 1, 6, 192, 320))


def _round_filters(f, width, divisor=8):
    f *= width
    new = max(divisor, int(f + divisor / 2) // divisor * divisor)
    if new < 0.9 * f:
        new += divisor
    return int(new)


class Conv2dStaticSamePadding(nn.Conv2d):
    """TF "SAME" padding computed once for the pretraining ``image_size`` (EfficientNet-PyTorch):
    the padding amounts are fixed at construction, whatever the input size later is."""

    def __init__(self, cin, cout, k, stride=1, groups=1, bias=False, image_size=None):
        super().__init__(cin, cout, k, stride, 0, groups=groups, bias=bias)
        ih = iw = image_size
        kh, kw = self.weight.shape[-2:]
        sh, sw = self.stride
        oh, ow = math.ceil(ih / sh), math.ceil(iw / sw)
        ph = max((oh - 1) * sh + kh - ih, 0)
        pw = max((ow - 1) * sw + kw - iw, 0)
        self._pad = (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2)
        self.static_padding = nn.ZeroPad2d(self._pad) if ph > 0 or pw > 0 else nn.Identity()

    def forward(self, x):
        l, r, t, b = self._pad
        if l == r and t == b:  # symmetric: the conv's own padding (no padded copy of x)
            return F.conv2d(x, self.weight, self.bias, self.stride, (t, l), self.dilation, self.groups)
        return F.conv2d(self.static_padding(x), self.weight, self.bias, self.stride, 0, self.dilation, self.groups)


class MBConvBlock(nn.Module):
    def __init__(self, cin, cout, k, stride, expand, image_size, se_ratio=0.25, bn_mom=0.01, bn_eps=1e-3):
        super().__init__()
        self.id_skip = stride == 1 and cin == cout
        oup = cin * expand
        if expand != 1:
            self._expand_conv = Conv2dStaticSamePadding(cin, oup, 1, image_size=image_size)
            self._bn0 = nn.BatchNorm2d(oup, momentum=bn_mom, eps=bn_eps)
        self.expand = expand
        self._depthwise_conv = Conv2dStaticSamePadding(oup, oup, k, stride, groups=oup, image_size=image_size)
        self._bn1 = nn.BatchNorm2d(oup, momentum=bn_mom, eps=bn_eps)
        sq = max(1, int(cin * se_ratio))
        self._se_reduce = Conv2dStaticSamePadding(oup, sq, 1, bias=True, image_size=1)
        self._se_expand = Conv2dStaticSamePadding(sq, oup, 1, bias=True, image_size=1)
        self._project_conv = Conv2dStaticSamePadding(oup, cout, 1, image_size=image_size)
        self._bn2 = nn.BatchNorm2d(cout, momentum=bn_mom, eps=bn_eps)

    def forward(self, inputs, drop_connect_rate=None):
        x = inputs
        if self.expand != 1:
            x = F.silu(self._bn0(self._expand_conv(x)))
        x = F.silu(self._bn1(self._depthwise_conv(x)))
        s = F.adaptive_avg_pool2d(x, 1)
        s = self._se_expand(F.silu(self._se_reduce(s)))
        x = ops.gate(x, s, sigmoid=True)  # sigmoid(s) * x in one pass
        x = self._bn2(self._project_conv(x))
        if self.id_skip:
            if drop_connect_rate and self.training:
                keep = 1.0 - drop_connect_rate
                mask = torch.floor(keep + torch.rand(x.shape[0], 1, 1, 1, dtype=x.dtype, device=x.device))
                x = x / keep * mask
            x = x + inputs
        return x


class EfficientNetEncoder(_EncoderMixin, nn.Module):
    """EfficientNet-PyTorch ``efficientnet-b*`` (keys ``_conv_stem``, ``_bn0``, ``_blocks.N.*``,
    ``_conv_head``, ``_bn1``), ``_fc`` removed -- SMP's ``EfficientNetEncoder``."""

    def __init__(self, name, depth=5):
        super().__init__()
        width, dep, res, _ = EFFNET_PARAMS[name]
        self._stage_idxs, chans = _EFFNET_SMP[name]
        self._drop_connect_rate = 0.2
        img = res
        stem = _round_filters(32, width)
        self._conv_stem = Conv2dStaticSamePadding(3, stem, 3, 2, image_size=img)
        self._bn0 = nn.BatchNorm2d(stem, momentum=0.01, eps=1e-3)
        img = math.ceil(img / 2)
        blocks = []
        for rep, k, s, e, i, o in _EFFNET_BLOCKS:
            cin, cout, n = _round_filters(i, width), _round_filters(o, width), int(math.ceil(dep * rep))
            blocks.append(MBConvBlock(cin, cout, k, s, e, img))
            img = math.ceil(img / s)
            for _ in range(n - 1):
                blocks.append(MBConvBlock(cout, cout, k, 1, e, img))
        self._blocks = nn.ModuleList(blocks)
        head = _round_filters(1280, width)
        self._conv_head = Conv2dStaticSamePadding(cout, head, 1, image_size=img)
        self._bn1 = nn.BatchNorm2d(head, momentum=0.01, eps=1e-3)
        self._set_channels(chans, depth)

    def get_stages(self):
        i = self._stage_idxs
        return [nn.Identity(), nn.Sequential(self._conv_stem, self._bn0),
                self._blocks[: i[0]], self._blocks[i[0]: i[1]], self._blocks[i[1]: i[2]], self._blocks[i[2]:]]

    def make_dilated(self, output_stride):
        if output_stride == 32:
            return
        # SMP: the depth-wise convs of the last stage(s) get dilation instead of stride
        plan = ((5, 2),) if output_stride == 16 else ((4, 2), (5, 4))
        self._output_stride = output_stride
        stages = self.get_stages()
        for idx, rate in plan:
            for m in stages[idx].modules():
                if isinstance(m, nn.Conv2d) and m.kernel_size[0] > 1:
                    m.stride = (1, 1)
                    m.dilation = (rate, rate)
                    kh = m.kernel_size[0]
                    p = (kh // 2) * rate
                    if isinstance(m, Conv2dStaticSamePadding):
                        m._pad = (p, p, p, p)
                        m.static_padding = nn.ZeroPad2d(m._pad)

    def forward(self, x):
        feats = [x]
        if self._depth >= 1:
            x = F.silu(self._bn0(self._conv_stem(x)))
            feats.append(x)
        i = self._stage_idxs
        bounds = [(0, i[0]), (i[0], i[1]), (i[1], i[2]), (i[2], len(self._blocks))]
        nb = len(self._blocks)
        for lo, hi in bounds[: max(0, self._depth - 1)]:
            for b in range(lo, hi):
                x = self._blocks[b](x, self._drop_connect_rate * b / nb)
            feats.append(x)
        return feats


# ---------------------------------------------------------------------------------------- SENet
SENET_SPECS = {  # block, layers, groups, reduction, base width
    "se_resnet50": ("se_resnet", (3, 4, 6, 3), 1, 16, 64),
    "se_resnet101": ("se_resnet", (3, 4, 23, 3), 1, 16, 64),
    "se_resnet152": ("se_resnet", (3, 8, 36, 3), 1, 16, 64),
    "se_resnext50_32x4d": ("se_resnext", (3, 4, 6, 3), 32, 16, 4),
    "se_resnext101_32x4d": ("se_resnext", (3, 4, 23, 3), 32, 16, 4),
}


class SEModule(nn.Module):
    def __init__(self, channels, reduction):
        super().__init__()
        self.fc1 = nn.Conv2d(channels, channels // reduction, 1)
        self.relu = nn.ReLU(inplace=True)
        self.fc2 = nn.Conv2d(channels // reduction, channels, 1)
        self.sigmoid = nn.Sigmoid()

    def forward(self, x):
        s = self.fc2(self.relu(self.fc1(F.adaptive_avg_pool2d(x, 1))))
        return ops.gate(x, s, sigmoid=True)


class SEBottleneck(nn.Module):
    """Cadene's SEResNetBottleneck (stride on the first 1x1) / SEResNeXtBottleneck (stride on
    the grouped 3x3)."""
    expansion = 4

    def __init__(self, kind, inplanes, planes, groups, reduction, base_width, stride=1, downsample=None):
        super().__init__()
        if kind == "se_resnext":
            width = math.floor(planes * (base_width / 64)) * groups
            s1, s2 = 1, stride
        else:
            width, s1, s2 = planes, stride, 1
        self.conv1 = nn.Conv2d(inplanes, width, 1, s1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, s2, 1, groups=groups, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.se_module = SEModule(planes * 4, reduction)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        out = ops.conv_bn_act(x, self.conv1, self.bn1, "relu")
        out = ops.conv_bn_act(out, self.conv2, self.bn2, "relu")
        out = self.se_module(self.bn3(self.conv3(out)))
        res = self.downsample(x) if self.downsample is not None else x
        return torch.relu(out + res)


class SENetEncoder(_EncoderMixin, nn.Module):
    """pretrainedmodels' SENet (keys ``layer0.conv1``, ``layer0.bn1``, ``layerN.M.se_module.fc1``,
    ``layerN.0.downsample.{0,1}``), ``avg_pool`` / ``last_linear`` removed -- SMP's
    ``SENetEncoder``."""

    def __init__(self, name, depth=5):
        super().__init__()
        kind, layers, groups, reduction, base_width = SENET_SPECS[name]
        self.layer0 = nn.Sequential()
        self.layer0.add_module("conv1", nn.Conv2d(3, 64, 7, 2, 3, bias=False))
        self.layer0.add_module("bn1", nn.BatchNorm2d(64))
        self.layer0.add_module("relu1", nn.ReLU(inplace=True))
        self.layer0.add_module("pool", nn.MaxPool2d(3, 2, ceil_mode=True))
        self.inplanes = 64
        for i, (planes, n) in enumerate(zip((64, 128, 256, 512), layers)):
            stride = 1 if i == 0 else 2
            ds = None
            if stride != 1 or self.inplanes != planes * 4:
                ds = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride, bias=False),
                                   nn.BatchNorm2d(planes * 4))
            blocks = [SEBottleneck(kind, self.inplanes, planes, groups, reduction, base_width, stride, ds)]
            self.inplanes = planes * 4
            blocks += [SEBottleneck(kind, self.inplanes, planes, groups, reduction, base_width) for _ in range(n - 1)]
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
        self._set_channels((3, 64, 256, 512, 1024, 2048), depth)

    def get_stages(self):
        return [nn.Identity(), self.layer0[:-1], nn.Sequential(self.layer0[-1], self.layer1),
                self.layer2, self.layer3, self.layer4]

    def _stage_fns(self):
        l0 = self.layer0
        return [lambda x: ops.conv_bn_act(x, l0.conv1, l0.bn1, "relu"),
                lambda x: self.layer1(l0.pool(x)), self.layer2, self.layer3, self.layer4]


EXTRA_ENCODERS = tuple(VGG_SPECS) + tuple(DENSENET_SPECS) + tuple(EFFNET_PARAMS) + tuple(SENET_SPECS)


def build_extra_encoder(name, depth=5):
    if name in VGG_SPECS:
        return VGGEncoder(name, depth)
    if name in DENSENET_SPECS:
        return DenseNetEncoder(name, depth)
    if name in EFFNET_PARAMS:
        return EfficientNetEncoder(name, depth)
    if name in SENET_SPECS:
        return SENetEncoder(name, depth)
    return None
