"""Lite-HRNet (arXiv:2104.06403) -- lightweight high-resolution network.

Parity target: reference models/lite_hrnet.py (LiteHRNet :15-47, StageBlock
:50-94, RepresentationHead :97-121, ShuffleBlock :124-156, CCWBlock :159-194
(conditional channel weighting), CrossResolutionWeightModule :197-223,
FusionBlock :226-298, SpatialWeightModule :301-315, Up/DownsampleBlock
:318-344).  Multi-resolution fusion runs as one accumulation per output
branch; every bilinear upsample in it is a fused resize+add kernel.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .modules import ConvBNAct, DSConvBNAct, DWConvBNAct, channel_shuffle, conv1x1

ARCHS = {"litehrnet18": (2, 4, 2), "litehrnet30": (3, 8, 3)}


class LiteHRNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, base_ch=40, arch_type="litehrnet18", repeat=2, act_type="relu"):
        super().__init__()
        if arch_type not in ARCHS:
            raise ValueError(f"Unsupport architecture type: {arch_type}.\n")
        mods = ARCHS[arch_type]
        self.stem = nn.Sequential(ConvBNAct(n_channel, 32, 3, 2, act_type=act_type),
                                  ShuffleBlock(32, base_ch, 2, act_type))
        self.stage1_down = DSConvBNAct(base_ch, base_ch * 2, 3, 2, act_type=act_type)
        self.stage2 = StageBlock(base_ch, 2, repeat, mods[0], act_type)
        self.stage3 = StageBlock(base_ch, 3, repeat, mods[1], act_type)
        self.stage4 = StageBlock(base_ch, 4, repeat, mods[2], act_type)
        self.rep_head = RepresentationHead(base_ch, num_class, 4, act_type)

    def forward(self, x, is_training=False):
        s = self.stem(x)
        feats = [s, self.stage1_down(s)]
        feats = self.stage4(self.stage3(self.stage2(feats)))
        return ops.final_upsample(self.rep_head(feats), x.shape[2:], True)


class StageBlock(nn.Module):
    def __init__(self, base_ch, stage, repeat, num_modules, act_type):
        super().__init__()
        if stage < 2 or repeat <= 0 or num_modules <= 0:
            raise AssertionError
        chs = [2 ** i * base_ch for i in range(stage)]
        blocks = []
        for i in range(num_modules):
            blocks.append(CrossResolutionWeightModule(sum(chs) // 2, act_type))
            blocks.append(nn.ModuleList([nn.ModuleList([CCWBlock(c, c, 1, act_type) for _ in range(repeat)])
                                         for c in chs]))
            blocks.append(FusionBlock(base_ch, stage, i == num_modules - 1 and stage != 4, act_type))
        self.stage_blocks = nn.ModuleList(blocks)

    def forward(self, feats):
        feats = list(feats)
        for i in range(0, len(self.stage_blocks), 3):
            crw, ccw, fusion = self.stage_blocks[i], self.stage_blocks[i + 1], self.stage_blocks[i + 2]
            w = crw(feats)
            for j, chain in enumerate(ccw):
                for m in chain:
                    feats[j] = m(feats[j], w[j])
            feats = fusion(feats)
        return feats


class RepresentationHead(nn.Module):
    def __init__(self, base_ch, num_class, num_stage, act_type, hid_ch=128):
        super().__init__()
        self.up = nn.ModuleList([nn.Identity()] + [nn.Upsample(scale_factor=2 ** (i + 1), mode="bilinear",
                                                               align_corners=True) for i in range(num_stage - 1)])
        in_ch = sum(2 ** i for i in range(num_stage)) * base_ch
        self.seg_head = nn.Sequential(DSConvBNAct(in_ch, hid_ch, 3, act_type=act_type), conv1x1(hid_ch, num_class))

    def forward(self, feats):
        hw = feats[0].shape[2:]
        ups = [feats[0]] + [ops.interpolate(f, (f.shape[2] * m.scale_factor, f.shape[3] * m.scale_factor), True)
                            for f, m in zip(feats[1:], list(self.up)[1:])]
        return self.seg_head(torch.cat(ups, dim=1))


class ShuffleBlock(nn.Module):
    def __init__(self, in_channels, out_channels, stride, act_type):
        super().__init__()
        if stride not in (1, 2):
            raise AssertionError
        il, ol = in_channels // 2, out_channels // 2
        ir, orr = in_channels - il, out_channels - ol
        self.in_ch_l = il
        self.left_branch = (ConvBNAct(il, ol, 1, stride, act_type=act_type) if stride != 1 or il != ol
                            else nn.Identity())
        self.right_branch = nn.Sequential(ConvBNAct(ir, orr, 1, act_type=act_type),
                                          DWConvBNAct(orr, orr, 3, stride, act_type=act_type),
                                          ConvBNAct(orr, orr, 1, act_type=act_type))

    def forward(self, x):
        c = self.in_ch_l
        return channel_shuffle(torch.cat([self.left_branch(x[:, :c]), self.right_branch(x[:, c:])], dim=1))


class CCWBlock(nn.Module):
    """Conditional channel weighting: cross-resolution weights before the DW conv, spatial weights after."""

    def __init__(self, in_channels, out_channels, stride, act_type):
        super().__init__()
        if stride not in (1, 2):
            raise AssertionError
        il, ol = in_channels // 2, out_channels // 2
        ir, orr = in_channels - il, out_channels - ol
        self.split_ch = [il, ir]
        self.left_branch = (ConvBNAct(il, ol, 1, stride, act_type=act_type) if stride != 1 or il != ol
                            else nn.Identity())
        self.right_branch = DWConvBNAct(ir, orr, 3, stride, act_type=act_type)
        self.sw = SpatialWeightModule(orr, act_type)

    def forward(self, feats, cr_weight):
        fl, fr = torch.split(feats, self.split_ch, dim=1)
        if cr_weight.shape[2:] != fr.shape[2:]:
            cr_weight = F.interpolate(cr_weight, fr.shape[2:], mode="nearest")
        fr = self.right_branch(ops.gate(fr, cr_weight))
        fr = ops.gate(fr, self.sw(fr))
        return channel_shuffle(torch.cat([self.left_branch(fl), fr], dim=1))


class CrossResolutionWeightModule(nn.Module):
    def __init__(self, channels, act_type, ch_reduction=8, pool_size=None):
        super().__init__()
        hid = channels // ch_reduction
        self.pool_size = pool_size
        self.conv = nn.Sequential(ConvBNAct(channels, hid, 1, act_type=act_type),
                                  ConvBNAct(hid, channels, 1, act_type="sigmoid"))

    def forward(self, feats):
        ps = feats[-1].shape[2:] if self.pool_size is None else self.pool_size
        halves = [f.shape[1] // 2 for f in feats]
        parts = [f[:, h:] if i == len(feats) - 1 else F.adaptive_avg_pool2d(f[:, h:], ps)
                 for i, (f, h) in enumerate(zip(feats, halves))]
        return torch.split(self.conv(torch.cat(parts, dim=1)), halves, dim=1)


class FusionBlock(nn.Module):
    """Exchange between resolutions: output i = sum_j stream_{j+1}[i](feats[j])."""

    def __init__(self, base_ch, stage, extra_output, act_type):
        super().__init__()
        if stage not in (2, 3, 4):
            raise AssertionError
        self.stage, self.extra_output = stage, extra_output
        n_out = stage + 1 if extra_output else stage
        ch = [2 ** i * base_ch for i in range(n_out)]
        self.stream1 = nn.ModuleList([nn.Identity()] + [DownsampleBlock(ch[0], ch[i], i, act_type)
                                                        for i in range(1, n_out)])
        self.stream2 = nn.ModuleList([UpsampleBlock(ch[1], ch[0], 2, act_type), nn.Identity()]
                                     + [DownsampleBlock(ch[1], ch[i + 1], i, act_type) for i in range(1, n_out - 1)])
        if stage in (3, 4):
            s3 = [UpsampleBlock(ch[2], ch[2 - i], 2 ** i, act_type) for i in (2, 1)] + [nn.Identity()]
            if extra_output or stage == 4:
                s3.append(DownsampleBlock(ch[2], ch[3], 1, act_type))
            self.stream3 = nn.ModuleList(s3)
        if stage == 4:
            self.stream4 = nn.ModuleList([UpsampleBlock(ch[3], ch[3 - i], 2 ** i, act_type) for i in (3, 2, 1)]
                                         + [nn.Identity()])

    def forward(self, feats):
        if len(feats) != self.stage:
            raise AssertionError
        streams = [self.stream1, self.stream2]
        if self.stage >= 3:
            streams.append(self.stream3)
        if self.stage == 4:
            streams.append(self.stream4)
        outs = []
        for i in range(len(self.stream1)):
            acc = None
            for j, stream in enumerate(streams):
                m = stream[i]
                if isinstance(m, UpsampleBlock):
                    y = m[0](feats[j])
                    s = m[1].scale_factor
                    acc = ops.interpolate(y, (y.shape[2] * s, y.shape[3] * s), True, skip=acc)
                else:
                    y = m(feats[j])
                    acc = y if acc is None else acc + y
            outs.append(acc)
        return outs


class SpatialWeightModule(nn.Module):
    def __init__(self, channels, act_type, ch_reduction=8):
        super().__init__()
        hid = channels // ch_reduction
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Sequential(ConvBNAct(channels, hid, 1, act_type=act_type),
                                ConvBNAct(hid, channels, 1, act_type="sigmoid"))

    def forward(self, x):
        return self.fc(self.avg_pool(x))


class UpsampleBlock(nn.Sequential):
    def __init__(self, in_ch, out_ch, scale_factor, act_type):
        super().__init__(ConvBNAct(in_ch, out_ch, 1, act_type=act_type),
                         nn.Upsample(scale_factor=scale_factor, mode="bilinear", align_corners=True))


class DownsampleBlock(nn.Module):
    def __init__(self, in_ch, out_ch, num_block, act_type):
        super().__init__()
        if num_block < 1:
            raise AssertionError
        self.conv = nn.Sequential(*[DSConvBNAct(in_ch, in_ch if i != num_block - 1 else out_ch, 3, 2,
                                                act_type=act_type) for i in range(num_block)])

    def forward(self, x):
        return self.conv(x)
