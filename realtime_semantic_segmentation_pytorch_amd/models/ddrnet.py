"""DDRNet -- Deep Dual-resolution Networks (arXiv:2101.06085).

Parity target: reference models/ddrnet.py (DDRNet :16-63 with arch table :20-23,
Stage2-5 :66-165, RB :168-191, RBB :194-219, BilateralFusion :222-238,
DAPPM :241-291).  Attribute names match the reference so ``state_dict`` keys are
interchangeable (306 keys for DDRNet-23 with aux head).

MI355X notes: every "upsample low-res branch and add into the high-res branch"
site (bilateral fusion, DAPPM cascade, stage-5 merge) is one fused HIP kernel
``ops.interpolate(x, size, skip=..., act=...)`` instead of interpolate + add +
activation, and the final logit upsample goes through ``ops.final_upsample`` so
the training loss can consume the 1/8-resolution logits directly.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .modules import Activation, ConvBNAct, SegHead, conv1x1

ARCHS = {
    # name: (base channels, blocks per stage: s2, s3, s4a, s4b, s5a, s5b)
    "DDRNet-23-slim": (32, (2, 2, 2, 0, 2, 1)),
    "DDRNet-23": (64, (2, 2, 2, 0, 2, 1)),
    "DDRNet-39": (64, (3, 4, 3, 3, 3, 1)),
}


def _fusable(act: Activation) -> bool:
    return act.act_type in ("relu", "relu6", "none")


def _resize_add_act(x_small, size, skip, act: Activation):
    """act(skip + bilinear(x_small -> size)), fused on GPU when the activation allows."""
    if _fusable(act):
        return ops.interpolate(x_small, size, True, skip=skip, act=act.act_type)
    return act(skip + ops.interpolate(x_small, size, True))


class DDRNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, arch_type="DDRNet-23-slim", act_type="relu",
                 use_aux=True):
        super().__init__()
        if arch_type not in ARCHS:
            raise ValueError(f"Unsupport architecture type: {arch_type}.\n")
        c, reps = ARCHS[arch_type]
        self.arch_type = arch_type
        self.use_aux = use_aux
        self.conv1 = ConvBNAct(n_channel, c, 3, 2, act_type=act_type)
        self.conv2 = Stage2(c, reps[0], act_type)
        self.conv3 = Stage3(c, reps[1], act_type)
        self.conv4 = Stage4(c, reps[2], reps[3], act_type)
        self.conv5 = Stage5(c, reps[4], reps[5], act_type)
        self.seg_head = SegHead(4 * c, num_class, act_type)
        if use_aux:
            self.aux_head = SegHead(2 * c, num_class, act_type)

    def forward(self, x, is_training=False):
        out_hw = x.shape[2:]
        x = self.conv3(self.conv2(self.conv1(x)))
        x_low, x_high = self.conv4(x)
        # the aux head only when it is returned (the reference evaluates it in inference too and
        # drops it: same outputs, ~4 kernels less per inference forward)
        aux = self.aux_head(x_high) if self.use_aux and is_training else None
        x = self.seg_head(self.conv5(x_low, x_high))
        x = ops.final_upsample(x, out_hw, True)
        if torch.onnx.is_in_onnx_export():
            return ops.materialize(x).argmax(1, keepdim=True).to(torch.int8)
        if self.use_aux and is_training:
            return x, (aux,)
        return x


def _stack(block, cin, cout, stride, n, act_type):
    """`n` blocks; only the first changes stride / width (reference build_blocks)."""
    layers = [block(cin, cout, stride, act_type=act_type)]
    layers += [block(cout, cout, 1, act_type=act_type) for _ in range(1, n)]
    return nn.Sequential(*layers)


class Stage2(nn.Module):
    def __init__(self, c, n, act_type="relu"):
        super().__init__()
        self.conv = nn.Sequential(ConvBNAct(c, c, 3, 2, act_type=act_type),
                                  *[RB(c, c, 1, act_type) for _ in range(n)])

    def forward(self, x):
        return self.conv(x)


class Stage3(nn.Module):
    def __init__(self, c, n, act_type="relu"):
        super().__init__()
        self.conv = _stack(RB, c, 2 * c, 2, n, act_type)

    def forward(self, x):
        return self.conv(x)


class Stage4(nn.Module):
    def __init__(self, c, n1, n2, act_type="relu"):
        super().__init__()
        lo, hi = 4 * c, 2 * c
        self.low_conv1 = _stack(RB, 2 * c, lo, 2, n1, act_type)
        self.high_conv1 = _stack(RB, 2 * c, hi, 1, n1, act_type)
        self.bilateral_fusion1 = BilateralFusion(lo, hi, 2)
        self.extra_conv = n2 > 0
        if self.extra_conv:
            self.low_conv2 = _stack(RB, lo, lo, 1, n2, act_type)
            self.high_conv2 = _stack(RB, hi, hi, 1, n2, act_type)
            self.bilateral_fusion2 = BilateralFusion(lo, hi, 2)

    def forward(self, x):
        # the two branches run concurrently in inference (ops/streams.py): batch-1 grids are small
        x_low, x_high = ops.concurrent_branches(lambda: self.low_conv1(x), lambda: self.high_conv1(x), x.device)
        x_low, x_high = self.bilateral_fusion1(x_low, x_high)
        if self.extra_conv:
            x_low, x_high = ops.concurrent_branches(lambda: self.low_conv2(x_low), lambda: self.high_conv2(x_high),
                                                    x.device)
            x_low, x_high = self.bilateral_fusion2(x_low, x_high)
        return x_low, x_high


class Stage5(nn.Module):
    def __init__(self, c, n1, n2, act_type="relu"):
        super().__init__()
        self.low_conv1 = _stack(RB, 4 * c, 8 * c, 2, n1, act_type)
        self.high_conv1 = _stack(RB, 2 * c, 2 * c, 1, n1, act_type)
        self.bilateral_fusion = BilateralFusion(8 * c, 2 * c, 4)
        self.low_conv2 = _stack(RBB, 8 * c, 16 * c, 2, n2, act_type)
        self.high_conv2 = _stack(RBB, 2 * c, 4 * c, 1, n2, act_type)
        self.dappm = DAPPM(16 * c, 4 * c)

    def forward(self, x_low, x_high):
        hw = x_high.shape[2:]
        dev = x_high.device
        x_low, x_high = ops.concurrent_branches(lambda: self.low_conv1(x_low), lambda: self.high_conv1(x_high), dev)
        x_low, x_high = self.bilateral_fusion(x_low, x_high)
        x_low, y_high = ops.concurrent_branches(lambda: self.dappm(self.low_conv2(x_low)),
                                                lambda: self.high_conv2(x_high), dev)
        # high_conv2(x_high) + upsample(x_low) in one kernel
        return ops.interpolate(x_low, hw, True, skip=y_high)


class RB(nn.Module):
    """Basic residual block (two 3x3), projection shortcut when shape changes."""

    def __init__(self, in_channels, out_channels, stride=1, act_type="relu"):
        super().__init__()
        self.downsample = stride > 1 or in_channels != out_channels
        self.conv1 = ConvBNAct(in_channels, out_channels, 3, stride, act_type=act_type)
        self.conv2 = ConvBNAct(out_channels, out_channels, 3, 1, act_type="none")
        if self.downsample:
            self.conv_down = ConvBNAct(in_channels, out_channels, 1, stride, act_type="none")
        self.act = nn.ReLU()

    def forward(self, x):
        if self.downsample:
            # conv1 and the projection shortcut read x: one autograd node, one input gradient
            hs = self.conv1.start_twin(self.conv_down, x)
            if hs is not None:
                return self.conv2(self.conv1.finish(hs[0]), residual=self.conv_down.finish(hs[1]), act=self.act)
        shortcut = self.conv_down(x) if self.downsample else x
        # relu(BN(conv2(.)) + shortcut) as one fused BN/residual/activation kernel
        return self.conv2(self.conv1(x), residual=shortcut, act=self.act)


class RBB(nn.Module):
    """Bottleneck residual block (1x1 -> 3x3 -> 1x1)."""

    def __init__(self, in_channels, out_channels, stride=1, act_type="relu"):
        super().__init__()
        self.downsample = stride > 1 or in_channels != out_channels
        self.conv1 = ConvBNAct(in_channels, in_channels, 1, act_type=act_type)
        self.conv2 = ConvBNAct(in_channels, in_channels, 3, stride, act_type=act_type)
        self.conv3 = ConvBNAct(in_channels, out_channels, 1, act_type="none")
        if self.downsample:
            self.conv_down = ConvBNAct(in_channels, out_channels, 1, stride, act_type="none")
        self.act = Activation(act_type)

    def forward(self, x):
        if self.downsample:
            hs = self.conv1.start_twin(self.conv_down, x)
            if hs is not None:
                return self.conv3(self.conv2(self.conv1.finish(hs[0])), residual=self.conv_down.finish(hs[1]),
                                  act=self.act)
        shortcut = self.conv_down(x) if self.downsample else x
        return self.conv3(self.conv2(self.conv1(x)), residual=shortcut, act=self.act)


class BilateralFusion(nn.Module):
    """Exchange between the low-res (semantic) and high-res (detail) branches."""

    def __init__(self, low_res_channels, high_res_channels, stride, act_type="relu"):
        super().__init__()
        self.conv_low = ConvBNAct(low_res_channels, high_res_channels, 1, act_type="none")
        self.conv_high = ConvBNAct(high_res_channels, low_res_channels, 3, stride, act_type="none")
        self.act = Activation(act_type)

    def forward(self, x_low, x_high):
        # both branch convs first, their SyncBN statistics all-reduces in flight together (each
        # overlaps the other branch's conv), then the two BN tails
        h_low = self.conv_high.start(x_high)
        h_high = self.conv_low.start(x_low)
        new_low = self.conv_high.finish(h_low, residual=x_low, act=self.act)
        new_high = _resize_add_act(self.conv_low.finish(h_high), x_high.shape[2:], x_high, self.act)
        return new_low, new_high


class DAPPM(nn.Module):
    """Deep Aggregation Pyramid Pooling Module (hierarchical pooled context)."""

    # (kernel, stride) of the average pools for branches 2..5; None = global pool
    POOLS = ((5, 2), (9, 4), (17, 8), None)

    def __init__(self, in_channels, out_channels, act_type="relu"):
        super().__init__()
        hid = in_channels // 4
        self.hid = hid
        self.conv0 = ConvBNAct(in_channels, out_channels, 1, act_type=act_type)
        self.conv1 = ConvBNAct(in_channels, hid, 1, act_type=act_type)
        for i, spec in enumerate(self.POOLS, start=2):
            pool = nn.AdaptiveAvgPool2d(1) if spec is None else nn.AvgPool2d(spec[0], spec[1], (spec[0] - 1) // 2)
            setattr(self, f"pool{i}", nn.Sequential(pool, conv1x1(in_channels, hid)))
            setattr(self, f"conv{i}", ConvBNAct(hid, hid, 3, act_type=act_type))
        self.conv_last = ConvBNAct(hid * 5, out_channels, 1, act_type=act_type)

    def forward(self, x):
        hw = x.shape[2:]
        # the five branches land in one concat buffer (ops/concat.py)
        sink = ops.ConcatSink([self.hid] * 5)
        # the pooled 1 x 1 projections do not depend on the chain: in inference they run on a side
        # stream while conv0 / conv1 run (ops/streams.py); in training they interleave as before
        (y0, prev), pooled = ops.concurrent_branches(
            lambda: (self.conv0(x), self.conv1(x, sink=(sink, 0))),
            lambda: [getattr(self, f"pool{i}")(x) for i in range(2, 6)], x.device)
        branches = [prev]
        for i in range(2, 6):
            prev = getattr(self, f"conv{i}")(ops.interpolate(pooled[i - 2], hw, True, skip=prev), sink=(sink, i - 1))
            branches.append(prev)
        return self.conv_last(sink.cat(branches)) + y0
