"""STDC-Seg -- "Rethinking BiSeNet for real-time semantic segmentation" (arXiv:2104.13188).

Parity target: reference models/stdc.py (STDC :16-101 with encoder_type
stdc1/stdc2, aux heads at 1/8, 1/16, 1/32 or a detail head; STDCModule
:104-128; LaplacianConv :131-147).  Key names match the reference.

MI355X notes: ARM attention runs on pooled vectors, the two "upsample x2 and
add" merges are fused resize-add kernels, the final resize is deferred to the
loss; ``LaplacianConv`` builds the 3-scale detail ground truth on device.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .bisenetv1 import AttentionRefinementModule, FeatureFusionModule
from .modules import ConvBNAct, SegHead, conv1x1

STDC_REPEATS = {"stdc1": (1, 1, 1), "stdc2": (3, 4, 2)}


def _up2(x, skip=None):
    return ops.interpolate(x, (x.shape[2] * 2, x.shape[3] * 2), True, skip=skip)


class STDC(nn.Module):
    def __init__(self, num_class=1, n_channel=3, encoder_type="stdc1", use_detail_head=False,
                 use_aux=False, act_type="relu"):
        super().__init__()
        if encoder_type not in STDC_REPEATS:
            raise ValueError("Unsupported encoder type.\n")
        if use_detail_head and use_aux:
            raise AssertionError("Currently only support either aux-head or detail head.\n")
        reps = STDC_REPEATS[encoder_type]
        self.use_detail_head, self.use_aux = use_detail_head, use_aux
        self.stage1 = ConvBNAct(n_channel, 32, 3, 2)
        self.stage2 = ConvBNAct(32, 64, 3, 2)
        self.stage3 = self._make_stage(64, 256, reps[0], act_type)
        self.stage4 = self._make_stage(256, 512, reps[1], act_type)
        self.stage5 = self._make_stage(512, 1024, reps[2], act_type)
        if use_aux:
            self.aux_head3 = SegHead(256, num_class, act_type)
            self.aux_head4 = SegHead(512, num_class, act_type)
            self.aux_head5 = SegHead(1024, num_class, act_type)
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.arm4 = AttentionRefinementModule(512)
        self.arm5 = AttentionRefinementModule(1024)
        self.conv4 = conv1x1(512, 256)
        self.conv5 = conv1x1(1024, 256)
        self.ffm = FeatureFusionModule(256 + 256, 128, act_type)
        self.seg_head = SegHead(128, num_class, act_type)
        if use_detail_head:
            self.detail_head = SegHead(256, 1, act_type)
            self.detail_conv = conv1x1(3, 1)

    @staticmethod
    def _make_stage(cin, cout, repeats, act_type):
        return nn.Sequential(STDCModule(cin, cout, 2, act_type),
                             *[STDCModule(cout, cout, 1, act_type) for _ in range(repeats)])

    def forward(self, x, is_training=False):
        out_hw = x.shape[2:]
        x = self.stage2(self.stage1(x))
        x3 = self.stage3(x)
        x4 = self.stage4(x3)
        x5 = self.stage5(x4)
        aux = (self.aux_head3(x3), self.aux_head4(x4), self.aux_head5(x5)) if self.use_aux and is_training else ()
        x5 = self.conv5(self.pool(x5) + self.arm5(x5))
        x4 = _up2(_up2(x5, skip=self.conv4(self.arm4(x4))))
        x = self.seg_head(self.ffm(x4, x3))
        x = ops.final_upsample(x, out_hw, True)
        if torch.onnx.is_in_onnx_export():
            return ops.materialize(x).argmax(1, keepdim=True).to(torch.int8)
        if self.use_detail_head and is_training:
            return x, self.detail_head(x3)
        if self.use_aux and is_training:
            return x, aux
        return x


class STDCModule(nn.Module):
    """Short-term dense concatenation: 1x1 -> 3x3 (stride) -> 3x3 -> 3x3, widths C/2, C/4, C/8, C/8."""

    def __init__(self, in_channels, out_channels, stride, act_type):
        super().__init__()
        if out_channels % 8:
            raise ValueError("Output channel should be evenly divided by 8.\n")
        if stride not in (1, 2):
            raise ValueError(f"Unsupported stride: {stride}\n")
        self.stride = stride
        self.widths = [out_channels // 2, out_channels // 4, out_channels // 8, out_channels // 8]
        self.block1 = ConvBNAct(in_channels, out_channels // 2, 1)
        self.block2 = ConvBNAct(out_channels // 2, out_channels // 4, 3, stride)
        if stride == 2:
            self.pool = nn.AvgPool2d(3, 2, 1)
        self.block3 = ConvBNAct(out_channels // 4, out_channels // 8, 3)
        self.block4 = ConvBNAct(out_channels // 8, out_channels // 8, 3)

    def forward(self, x):
        # the four branches land in one concat buffer (ops/concat.py): their BN kernels store
        # there too, and the cat's backward hands each BN its gradient slice in place
        sink = ops.ConcatSink(self.widths)
        x1 = self.block1(x, sink=(sink, 0) if self.stride == 1 else None)
        x2 = self.block2(x1, sink=(sink, 1))
        if self.stride == 2:
            x1 = self.pool(x1)
        x3 = self.block3(x2, sink=(sink, 2))
        return sink.cat([x1, x2, x3, self.block4(x3, sink=(sink, 3))])


class LaplacianConv(nn.Module):
    """3-scale Laplacian edge map of a label image (detail ground truth), [N,1,H,W] -> [N,3,H,W]."""

    def __init__(self, device=None):
        super().__init__()
        k = torch.full((1, 1, 3, 3), -1.0)
        k[0, 0, 1, 1] = 8.0
        self.register_buffer("laplacian_kernel", k.to(device) if device is not None else k)

    def forward(self, lbl):
        k = self.laplacian_kernel.to(device=lbl.device, dtype=lbl.dtype)
        hw = lbl.shape[2:]
        outs = [F.conv2d(lbl, k, stride=1, padding=1)]
        for s in (2, 4):
            outs.append(F.interpolate(F.conv2d(lbl, k, stride=s, padding=1), hw, mode="nearest"))
        return torch.cat(outs, dim=1)
