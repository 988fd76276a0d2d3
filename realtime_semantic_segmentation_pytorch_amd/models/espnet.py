"""ESPNet (arXiv:1803.06815) -- efficient spatial pyramid of dilated convolutions.

Parity target: reference models/espnet.py (ESPNet :15-68 with the four
variants espnet / -a / -b / -c, L2Block :71-107, L3Block :110-149, Decoder
:152-179, ESPModule :182-235 -- reduce, K dilated branches, hierarchical sum,
concat, residual).  The reference mutates its ``block_channel`` default list
for espnet-a; here the list is copied.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .modules import ConvBNAct, DeConvBNAct, conv1x1

ARCH_TYPES = ("espnet", "espnet-a", "espnet-b", "espnet-c")


class ESPNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, arch_type="espnet", K=5, alpha2=2, alpha3=8,
                 block_channel=(16, 64, 128), act_type="prelu"):
        super().__init__()
        if arch_type not in ARCH_TYPES:
            raise ValueError(f"Unsupport architecture type: {arch_type}.\n")
        self.arch_type = arch_type
        self.use_skip = arch_type in ("espnet", "espnet-b", "espnet-c")
        self.reinforce = arch_type in ("espnet", "espnet-c")
        self.use_decoder = arch_type == "espnet"
        bc = list(block_channel)
        if arch_type == "espnet-a":
            bc[2] = bc[1]
        self.l1_block = ConvBNAct(n_channel, bc[0], 3, 2, act_type=act_type)
        self.l2_block = L2Block(bc[0], bc[1], arch_type, alpha2, self.use_skip, self.reinforce, act_type)
        self.l3_block = L3Block(bc[2], num_class, arch_type, alpha3, self.use_skip, self.reinforce,
                                self.use_decoder, act_type)
        if self.use_decoder:
            self.decoder = Decoder(num_class, 19, 131, act_type)

    def forward(self, x, is_training=False):
        img = x
        y = self.l1_block(x)
        if self.reinforce:  # input reinforcement: image resized (align_corners=False) to each level
            # (autocast: the fp32 image joins in the features' dtype instead of promoting them)
            y = torch.cat([y, ops.interpolate(img, y.shape[2:], False).to(y.dtype)], dim=1)
            y_l1 = y
            y = self.l2_block(y, img)
            y_l2 = y
        else:
            y = self.l2_block(y)
        y = self.l3_block(y)
        if self.use_decoder:
            return self.decoder(y, y_l1, y_l2)
        return ops.final_upsample(y, img.shape[2:], True)


class L2Block(nn.Module):
    def __init__(self, in_channels, hid_channels, arch_type, alpha, use_skip, reinforce, act_type="prelu"):
        super().__init__()
        self.arch_type, self.alpha, self.use_skip, self.reinforce = arch_type, alpha, use_skip, reinforce
        self.conv1 = ESPModule(in_channels + (3 if reinforce else 0), hid_channels, stride=2, act_type=act_type)
        self.layers = nn.Sequential(*[ESPModule(hid_channels, hid_channels, act_type=act_type) for _ in range(alpha)])

    def forward(self, x, x_input=None):
        s = self.conv1(x)
        y = self.layers(s)
        if self.use_skip:
            y = torch.cat([y, s], dim=1)
        if self.reinforce:
            y = torch.cat([y, ops.interpolate(x_input, y.shape[2:], False).to(y.dtype)], dim=1)
        return y


class L3Block(nn.Module):
    def __init__(self, in_channels, out_channels, arch_type, alpha, use_skip, reinforce, use_decoder,
                 act_type="prelu"):
        super().__init__()
        self.arch_type, self.alpha, self.use_skip = arch_type, alpha, use_skip
        self.conv1 = ESPModule(in_channels + (3 if reinforce else 0), 128, stride=2, act_type=act_type)
        self.layers = nn.Sequential(*[ESPModule(128, 128, act_type=act_type) for _ in range(alpha)])
        if use_decoder:
            self.conv_last = ConvBNAct(256, out_channels, 1, act_type=act_type)
        else:
            self.conv_last = conv1x1(256 if use_skip else 128, out_channels)

    def forward(self, x):
        s = self.conv1(x)
        y = self.layers(s)
        if self.use_skip:
            y = torch.cat([y, s], dim=1)
        return self.conv_last(y)


class Decoder(nn.Module):
    def __init__(self, num_class, l1_channel, l2_channel, act_type="prelu"):
        super().__init__()
        c = num_class
        self.upconv_l3 = DeConvBNAct(c, c, act_type=act_type)
        self.conv_cat_l2 = ConvBNAct(l2_channel, c, 1)
        self.conv_l2 = ESPModule(2 * c, c)
        self.upconv_l2 = DeConvBNAct(c, c, act_type=act_type)
        self.conv_cat_l1 = ConvBNAct(l1_channel, c, 1)
        self.conv_l1 = ESPModule(2 * c, c)
        self.upconv_l1 = DeConvBNAct(c, c)

    def forward(self, x, x_l1, x_l2):
        y = self.conv_l2(torch.cat([self.upconv_l3(x), self.conv_cat_l2(x_l2)], dim=1))
        y = self.conv_l1(torch.cat([self.upconv_l2(y), self.conv_cat_l1(x_l1)], dim=1))
        return self.upconv_l1(y)


class ESPModule(nn.Module):
    """Reduce (1x1, stride) -> K parallel 3x3 convs with dilation 2^k -> hierarchical sum -> concat."""

    def __init__(self, in_channels, out_channels, K=5, ks=3, stride=1, act_type="prelu"):
        super().__init__()
        self.K, self.stride = K, stride
        self.use_skip = in_channels == out_channels and stride == 1
        ckn = out_channels // K
        ck1 = out_channels - (K - 1) * ckn
        self.perfect_divisor = ck1 == ckn
        self.conv_kn = conv1x1(in_channels, ckn, stride)
        if not self.perfect_divisor:
            self.conv_k1 = conv1x1(in_channels, ck1, stride)
        self.layers = nn.ModuleList([ConvBNAct(ck1 if k == 0 else ckn, ck1 if k == 0 else ckn, ks, 1, 2 ** k,
                                               act_type=act_type) for k in range(K)])

    def forward(self, x):
        rn = self.conv_kn(x)
        r1 = rn if self.perfect_divisor else self.conv_k1(x)
        feats = [self.layers[0](r1)]
        # the first branch only joins the running sum when its width matches
        run = feats[0] if self.perfect_divisor else None
        for i in range(1, self.K):
            f = self.layers[i](rn)
            run = f if run is None else f + run
            feats.append(run)
        y = torch.cat(feats, dim=1)
        return y + x if self.use_skip else y
