"""BiSeNet V2 -- bilateral network with guided aggregation (arXiv:2004.02147).

Parity target: reference models/bisenetv2.py (BiSeNetv2 :17-40, DetailBranch
:43-54, SemanticBranch :57-106 with 4 aux SegHeads, StemBlock :109-127,
GatherExpansionLayer :130-162, ContextEmbeddingBlock :165-181,
BilateralGuidedAggregationLayer :184-221).  Module names match the reference
(360 state_dict keys with aux heads).

MI355X notes: the GE-layer residual ``act(shortcut + PW-BN(...))`` is one
fused BN/residual/ReLU kernel, the BGA ``x_high + upsample(x_low)`` one fused
resize-add kernel, and the final logit resize is deferred to the loss.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .modules import Activation, ConvBNAct, DWConvBNAct, PWConvBNAct, SegHead, conv1x1, conv3x3


class BiSeNetv2(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="relu", use_aux=True):
        super().__init__()
        self.use_aux = use_aux
        self.detail_branch = DetailBranch(n_channel, 128, act_type)
        self.semantic_branch = SemanticBranch(n_channel, 128, num_class, act_type, use_aux)
        self.bga_layer = BilateralGuidedAggregationLayer(128, 128, act_type)
        self.seg_head = SegHead(128, num_class, act_type)

    def forward(self, x, is_training=False):
        out_hw = x.shape[2:]
        x_d = self.detail_branch(x)
        sem = self.semantic_branch(x, want_aux=is_training)  # aux heads only when returned
        x_s, aux = (sem[0], sem[1:]) if self.use_aux else (sem, ())
        x = self.seg_head(self.bga_layer(x_d, x_s))
        x = ops.final_upsample(x, out_hw, True)
        if self.use_aux and is_training:
            return x, tuple(aux)
        return x


class DetailBranch(nn.Sequential):
    """Wide, shallow 1/8-resolution path: (cin -> 64 -> 64) s2, (64 x2, ->128) s2, (128 x3) s2."""

    # (in, out, stride) per ConvBNAct
    PLAN = ((None, 64, 2), (64, 64, 1), (64, 64, 2), (64, 64, 1), (64, 128, 1), (128, 128, 2),
            (128, 128, 1), (128, None, 1))

    def __init__(self, in_channels, out_channels, act_type="relu"):
        layers = []
        for cin, cout, s in self.PLAN:
            layers.append(ConvBNAct(cin or in_channels, cout or out_channels, 3, s, act_type=act_type))
        super().__init__(*layers)


class SemanticBranch(nn.Sequential):
    """Narrow, deep path with optional aux heads after stages 2, 3, 4, 5."""

    def __init__(self, in_channels, out_channels, num_class, act_type="relu", use_aux=False):
        super().__init__()
        self.use_aux = use_aux
        ge = GatherExpansionLayer
        self.stage1to2 = StemBlock(in_channels, 16, act_type)
        self.stage3 = nn.Sequential(ge(16, 32, 2, act_type), ge(32, 32, 1, act_type))
        self.stage4 = nn.Sequential(ge(32, 64, 2, act_type), ge(64, 64, 1, act_type))
        self.stage5_1to4 = nn.Sequential(ge(64, 128, 2, act_type),
                                         *[ge(128, 128, 1, act_type) for _ in range(3)])
        self.stage5_5 = ContextEmbeddingBlock(128, out_channels, act_type)
        if use_aux:
            for i, c in zip((2, 3, 4, 5), (16, 32, 64, 128)):
                setattr(self, f"seg_head{i}", SegHead(c, num_class, act_type))

    def forward(self, x, want_aux=True):
        aux = []
        for i, stage in zip((2, 3, 4, 5), (self.stage1to2, self.stage3, self.stage4, self.stage5_1to4)):
            x = stage(x)
            if self.use_aux:
                aux.append(getattr(self, f"seg_head{i}")(x) if want_aux else None)
        x = self.stage5_5(x)
        return (x, *aux) if self.use_aux else x


class StemBlock(nn.Module):
    def __init__(self, in_channels, out_channels, act_type="relu"):
        super().__init__()
        self.conv_init = ConvBNAct(in_channels, out_channels, 3, 2, act_type=act_type)
        self.left_branch = nn.Sequential(
            ConvBNAct(out_channels, out_channels // 2, 1, act_type=act_type),
            ConvBNAct(out_channels // 2, out_channels, 3, 2, act_type=act_type))
        self.right_branch = nn.MaxPool2d(3, 2, 1)
        self.conv_last = ConvBNAct(out_channels * 2, out_channels, 3, 1, act_type=act_type)

    def forward(self, x):
        x = self.conv_init(x)
        # K11: both branches land in one concat buffer -- the left branch's BN kernel stores into
        # its slice, the max pool runs inside the cat node into the other (ops.ConcatSink): no
        # pooled tensor and no cat kernel in forward, no slice copies in backward
        c = x.shape[1]  # both branches keep conv_init's width
        sink = ops.ConcatSink([c, c])
        left = self.left_branch[1](self.left_branch[0](x), sink=(sink, 0))
        rp = self.right_branch
        return self.conv_last(sink.cat([left, sink.max_pool(1, x, rp.kernel_size, rp.stride, rp.padding)]))


class GatherExpansionLayer(nn.Module):
    """3x3 conv -> depth-wise expansion (x6) -> 1x1 projection, residual (strided: DW+PW shortcut)."""

    def __init__(self, in_channels, out_channels, stride, act_type="relu", expand_ratio=6):
        super().__init__()
        self.stride = stride
        hid = int(round(in_channels * expand_ratio))
        layers = [ConvBNAct(in_channels, in_channels, 3, act_type=act_type)]
        if stride == 2:
            layers += [DWConvBNAct(in_channels, hid, 3, 2, act_type="none"),
                       DWConvBNAct(hid, hid, 3, 1, act_type="none")]
            self.right_branch = nn.Sequential(
                DWConvBNAct(in_channels, in_channels, 3, 2, act_type="none"),
                PWConvBNAct(in_channels, out_channels, act_type="none"))
        else:
            layers.append(DWConvBNAct(in_channels, hid, 3, 1, act_type="none"))
        layers.append(PWConvBNAct(hid, out_channels, act_type="none"))
        self.left_branch = nn.Sequential(*layers)
        self.act = Activation(act_type)

    def forward(self, x):
        shortcut = self.right_branch(x) if self.stride == 2 else x
        h = x
        for layer in list(self.left_branch)[:-1]:
            h = layer(h)
        # act(shortcut + BN(PW(h))) as one fused kernel
        return self.left_branch[-1](h, residual=shortcut, act=self.act)


class ContextEmbeddingBlock(nn.Module):
    def __init__(self, in_channels, out_channels, act_type="relu"):
        super().__init__()
        self.pool = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.BatchNorm2d(in_channels))
        self.conv_mid = ConvBNAct(in_channels, in_channels, 1, act_type=act_type)
        self.conv_last = conv3x3(in_channels, out_channels)

    def forward(self, x):
        return self.conv_last(x + self.conv_mid(self.pool(x)))


class BilateralGuidedAggregationLayer(nn.Module):
    def __init__(self, in_channels, out_channels, act_type="relu"):
        super().__init__()
        c = in_channels
        self.detail_high = nn.Sequential(DWConvBNAct(c, c, 3, act_type=act_type), conv1x1(c, c))
        self.detail_low = nn.Sequential(DWConvBNAct(c, c, 3, 2, act_type=act_type), nn.AvgPool2d(3, 2, 1))
        self.semantic_high = nn.Sequential(
            ConvBNAct(c, c, 3, act_type=act_type),
            nn.Upsample(scale_factor=4, mode="bilinear", align_corners=True), nn.Sigmoid())
        self.semantic_low = nn.Sequential(DWConvBNAct(c, c, 3, act_type=act_type), conv1x1(c, c),
                                          nn.Sigmoid())
        self.conv_last = ConvBNAct(c, out_channels, 3, act_type=act_type)

    def forward(self, x_d, x_s):
        s_high = self.semantic_high[0](x_s)
        s_high = ops.interpolate(s_high, (s_high.shape[2] * 4, s_high.shape[3] * 4), True)
        x_high = ops.gate(self.detail_high(x_d), s_high, sigmoid=True)  # * sigmoid(.), one pass
        s_low = self.semantic_low[1](self.semantic_low[0](x_s))
        x_low = ops.gate(self.detail_low(x_d), s_low, sigmoid=True)
        return self.conv_last(ops.interpolate(x_low, x_high.shape[2:], True, skip=x_high))
