"""ICNet (arXiv:1704.08545).

Parity target: reference models/icnet.py (ICNet :15-64 -- image cascade over
1/1, 1/2, 1/4 inputs with a shared dilated ResNet run twice;
CascadeFeatureFusionUnit :67-90 with optional aux classifiers;
HighResolutionBranch :93-99; the dilated ResNet wrapper :102-154 that turns the
first block of layer3 / layer4 into stride-1 dilation-2 / -4 convolutions).
"""
from __future__ import annotations

import torch.nn as nn

from .. import ops
from .backbone import ResNet as _TVResNet
from .modules import Activation, ConvBNAct, PyramidPoolingModule, SegHead


class ICNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, backbone_type="resnet18", act_type="relu", use_aux=True,
                 pretrained=False):
        super().__init__()
        if "resnet" not in backbone_type:
            raise NotImplementedError()
        self.backbone = ResNet(backbone_type, pretrained=pretrained)
        ch1, ch2 = self.backbone.out_channels[3], self.backbone.out_channels[1]
        self.use_aux = use_aux
        self.bottom_branch = HighResolutionBranch(n_channel, 128, act_type=act_type)
        self.ppm = PyramidPoolingModule(ch1, 256, act_type=act_type)
        self.cff42 = CascadeFeatureFusionUnit(256, ch2, 128, num_class, act_type, use_aux)
        self.cff21 = CascadeFeatureFusionUnit(128, 128, 128, num_class, act_type, use_aux)
        self.seg_head = SegHead(128, num_class, act_type)

    def forward(self, x, is_training=False):
        h, w = x.shape[2:]
        x_d2 = ops.interpolate(x, (h // 2, w // 2), True)
        x_d4 = ops.interpolate(x, (h // 4, w // 4), True)
        low = self.ppm(self.backbone(x_d4)[0])      # 1/32
        mid = self.backbone(x_d2)[1]                # 1/16
        high = self.bottom_branch(x)                # 1/8
        mid, aux2 = self.cff42(low, mid, is_training)  # aux classifiers only when returned
        high, aux3 = self.cff21(mid, high, is_training)
        y = self.seg_head(ops.interpolate(high, (high.shape[2] * 2, high.shape[3] * 2), True))
        y = ops.final_upsample(y, (h, w), True)
        if self.use_aux and is_training:
            return y, (aux2, aux3)
        return y


class CascadeFeatureFusionUnit(nn.Module):
    def __init__(self, channel1, channel2, out_channels, num_class, act_type, use_aux):
        super().__init__()
        self.use_aux = use_aux
        self.conv1 = ConvBNAct(channel1, out_channels, 3, 1, 2, act_type="none")
        self.conv2 = ConvBNAct(channel2, out_channels, 1, act_type="none")
        self.act = Activation(act_type)
        if use_aux:
            self.classifier = SegHead(channel1, num_class, act_type)

    def forward(self, x1, x2, want_aux=True):
        x1 = ops.interpolate(x1, (x1.shape[2] * 2, x1.shape[3] * 2), True)
        aux = self.classifier(x1) if self.use_aux and want_aux else None
        return self.conv2(x2, residual=self.conv1(x1), act=self.act), aux


class HighResolutionBranch(nn.Sequential):
    def __init__(self, in_channels, out_channels, hid_channels=32, act_type="relu"):
        widths = (in_channels, hid_channels, hid_channels * 2, out_channels)
        super().__init__(*[ConvBNAct(widths[i], widths[i + 1], 3, 2, act_type=act_type) for i in range(3)])


class ResNet(_TVResNet):
    """ResNet whose layer3[0] / layer4[0] keep resolution (stride 1) with dilation 2 / 4 in
    their strided conv -- only the first block of each stage, exactly like the reference
    wrapper; returns (layer4 output, layer2 output)."""

    def __init__(self, resnet_type, pretrained=False):
        super().__init__(resnet_type, pretrained=pretrained)
        basic = resnet_type in ("resnet18", "resnet34")
        for i, layer in ((1, self.layer3), (2, self.layer4)):
            blk = layer[0]
            old_down = blk.downsample[0]
            blk.downsample[0] = nn.Conv2d(old_down.in_channels, old_down.out_channels, 1, 1, bias=False)
            blk.downsample[0].weight.data.copy_(old_down.weight.data)
            old = blk.conv1 if basic else blk.conv2
            new = nn.Conv2d(old.in_channels, old.out_channels, 3, 1, 2 * i, 2 * i, bias=False)
            new.weight.data.copy_(old.weight.data)
            if basic:
                blk.conv1 = new
            else:
                blk.conv2 = new

    def forward(self, x):
        x2 = self.layer2(self.layer1(self.stem(x)))
        return self.layer4(self.layer3(x2)), x2
