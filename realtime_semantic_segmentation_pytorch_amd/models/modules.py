"""Building blocks shared by the model zoo.

Parity target: reference models/modules.py (conv3x3/conv1x1 :7-15,
channel_shuffle :18-32, DSConvBNAct :36-42, DWConvBNAct :46-59, PWConvBNAct
:63-69, ConvBNAct :73-85, DeConvBNAct :89-108, Activation :111-131,
PyramidPoolingModule :134-158, SegHead :161-166).

The module trees (and therefore ``state_dict`` keys such as ``<m>.0.weight``,
``<m>.1.running_mean``, ``<m>.2.activation.weight``, ``<m>.up_conv.0.weight``)
are kept identical to the reference so checkpoints interchange.  What differs
is the execution: resize/fusion points call the HIP kernels in
:mod:`..ops`, and ``ConvBNAct`` accepts ``groups`` (the reference lacks it, which
breaks RegSeg -- SURVEY A.1 #8).
"""
from __future__ import annotations

from typing import Sequence, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops

IntOrPair = Union[int, Sequence[int]]


def _same_padding(kernel_size: IntOrPair, dilation: int = 1):
    """'same' padding for odd kernels (int or (kh, kw)), scaled by dilation."""
    if isinstance(kernel_size, (list, tuple)):
        return tuple((k - 1) // 2 * dilation for k in kernel_size)
    return (kernel_size - 1) // 2 * dilation


def conv3x3(in_channels, out_channels, stride=1, bias=False):
    return nn.Conv2d(in_channels, out_channels, 3, stride, 1, bias=bias)


def conv1x1(in_channels, out_channels, stride=1, bias=False):
    return nn.Conv2d(in_channels, out_channels, 1, stride, 0, bias=bias)


def channel_shuffle(x: torch.Tensor, groups: int = 2) -> torch.Tensor:
    """ShuffleNet channel shuffle: [N, g*k, H, W] -> interleave the g groups (one HIP gather
    pass on GPU tensors, ``ops.channel_shuffle``)."""
    return ops.channel_shuffle(x, groups)


_ACTIVATIONS = {
    "relu": nn.ReLU, "relu6": nn.ReLU6, "leakyrelu": nn.LeakyReLU, "prelu": nn.PReLU,
    "celu": nn.CELU, "elu": nn.ELU, "hardswish": nn.Hardswish, "hardtanh": nn.Hardtanh,
    "gelu": nn.GELU, "glu": nn.GLU, "selu": nn.SELU, "silu": nn.SiLU, "sigmoid": nn.Sigmoid,
    "softmax": nn.Softmax, "tanh": nn.Tanh, "none": nn.Identity,
}


class Activation(nn.Module):
    """Named activation; the wrapped module lives at ``.activation`` (checkpoint ABI)."""

    def __init__(self, act_type: str, **kwargs):
        super().__init__()
        key = act_type.lower()
        if key not in _ACTIVATIONS:
            raise NotImplementedError(f"Unsupport activation type: {act_type}")
        self.act_type = key
        self.activation = _ACTIVATIONS[key](**kwargs)

    def forward(self, x):
        return self.activation(x)


class _FusedTail:
    """Mixin for ``Sequential(conv, bn, act)`` blocks: BN + (residual) + activation
    run as one fused HIP op (``ops.bn_act``) on channels-last GPU activations.

    ``forward(x, residual=None, act=None)`` computes
    ``act(own_act(bn(conv(x))) + residual)``; with a residual the block's own
    activation must be the identity (the reference's residual blocks are built
    that way: ``conv2`` of ``RB`` uses ``act_type='none'``).  ``sink=(ConcatSink, i)``:
    the output is branch ``i`` of a channel concat (ops/concat.py).
    """

    def forward(self, x, residual=None, act=None, sink=None):
        conv, bn, own = self[0], self[1], self[2]
        if ops.conv_ok(x, conv):
            y = self._mfma_tail(x, conv, bn, own, residual, act, sink)
            if y is not None:
                return y
        elif (residual is None and isinstance(conv, ops.DepthwiseConv2d)
              and isinstance(bn, (nn.BatchNorm2d, nn.SyncBatchNorm))
              and (bn.training or not bn.track_running_stats or bn.running_mean is None)):
            # depth-wise conv with the BN statistics in its epilogue (DWConvBNAct, K2)
            out = ops.dw_conv_bn_stats(x, conv)
            if out is not None:
                y, part = out
                return ops.bn_act(y, bn, own, act_module=own, part=part, sink=sink)
        elif residual is None and sink is None and isinstance(conv, ops.DepthwiseConv2d) and isinstance(
                bn, (nn.BatchNorm2d, nn.SyncBatchNorm)):
            # inference: the eval BN (+ ReLU / ReLU6) folded into the depth-wise kernel (one pass)
            code = ops.bn_act_code(own)
            y = ops.dw_conv_bn_eval(x, conv, bn, code) if code is not None else None
            if y is not None:
                return y
        y = ops.conv_forward(x, conv)
        if residual is None:
            return ops.bn_act(y, bn, own, act_module=own, sink=sink)
        own_code = ops.bn_act_code(own)
        if own_code != 0:  # own activation is not identity: apply it before the add
            y = ops.bn_act(y, bn, own, act_module=own)
            y = y + residual
            return act(y) if act is not None else y
        post = act if act is not None else "none"
        return ops.bn_act(y, bn, post, residual=residual,
                          act_module=act if isinstance(act, nn.Module) else None)

    def start(self, x):
        """First half of ``forward`` for a caller that interleaves independent branches: the conv
        with its BN statistics, whose SyncBN all-reduce is issued asynchronously
        (``ops.bn_stats_begin``); :meth:`finish` waits for it at the BN finalize.  Queued between
        the two, the other branch's conv overlaps the collective."""
        conv, bn = self[0], self[1]
        if (ops.conv_ok(x, conv) and isinstance(bn, (nn.BatchNorm2d, nn.SyncBatchNorm))
                and (bn.training or not bn.track_running_stats or bn.running_mean is None)):
            r = ops.conv_bn_stats(x, conv)
            if r is not None:
                y, part = r
                return y, part, ops.bn_stats_begin(y, bn, part)
        return (x,)

    def start_twin(self, other, x):
        """:meth:`start` of this block and of ``other`` (another conv + BN block reading the same
        ``x``, e.g. a downsampling residual block's projection shortcut) with both convs in one
        autograd node (``ops.twin_conv_bn_stats``): the input gradient is written once, with no
        accumulation add of the two.  None -> call :meth:`start` / ``forward`` separately."""
        blocks = (self, other)
        for b in blocks:
            bn = b[1]
            if not (isinstance(bn, (nn.BatchNorm2d, nn.SyncBatchNorm))
                    and (bn.training or not bn.track_running_stats or bn.running_mean is None)):
                return None
        if not (torch.is_grad_enabled() and x.requires_grad):
            return None  # nothing to save: the twin node only pays off in a training backward
        r = ops.twin_conv_bn_stats(x, self[0], other[0])
        if r is None:
            return None
        return tuple((y, part, ops.bn_stats_begin(y, b[1], part)) for b, (y, part) in zip(blocks, r))

    def finish(self, h, residual=None, act=None):
        """Second half of ``forward``: ``h`` from :meth:`start`."""
        if len(h) == 1:
            return self.forward(h[0], residual, act)
        y, part, pending = h
        bn, own = self[1], self[2]
        own_code = ops.bn_act_code(own)
        if residual is not None and own_code != 0:
            raise ValueError("start/finish: a residual needs the block's own activation to be identity")
        post = own_code if residual is None else (ops.bn_act_code(act) if act is not None else 0)
        return ops.bn_act(y, bn, post, residual=residual, part=part, pending=pending,
                          act_module=own if residual is None else (act if isinstance(act, nn.Module) else None))

    @staticmethod
    def _mfma_tail(x, conv, bn, own, residual, act, sink=None):
        """conv on the MFMA kernel with the BN statistics (training) or the whole
        BN + residual + activation tail (inference) in its epilogue; None -> stock path."""
        if not isinstance(bn, (nn.BatchNorm2d, nn.SyncBatchNorm)):
            return None
        own_code = ops.bn_act_code(own)
        if residual is None:
            post = own_code
        elif own_code == 0:
            post = ops.bn_act_code(act) if act is not None else 0
        else:
            return None
        if post is None:
            return None
        use_batch = bn.training or not bn.track_running_stats or bn.running_mean is None
        if not use_batch:
            return ops.conv_bn_act_eval(x, conv, bn, post, residual)
        # a stem whose BN recomputes the conv output from the image: no 2.1 GB store (ops/bn.py)
        store = not (residual is None and sink is None and post in (0, 1, 2)
                     and ops.stem_store_skippable(x, conv, bn))
        r = ops.conv_bn_stats(x, conv, store=store)
        if r is None:
            return None
        y, part = r
        return ops.bn_act(y, bn, post, residual=residual, part=part,
                          act_module=own if residual is None else (act if isinstance(act, nn.Module) else None),
                          sink=sink)


class ConvBNAct(_FusedTail, nn.Sequential):
    """Conv2d -> BatchNorm2d -> Activation, children ``0 / 1 / 2``."""

    def __init__(self, in_channels, out_channels, kernel_size: IntOrPair = 3, stride=1,
                 dilation=1, bias=False, act_type="relu", groups=1, **kwargs):
        conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride,
                         _same_padding(kernel_size, dilation), dilation, groups=groups, bias=bias)
        super().__init__(conv, nn.BatchNorm2d(out_channels), Activation(act_type, **kwargs))


class DWConvBNAct(_FusedTail, nn.Sequential):
    """Depth-wise conv (channel multiplier = out/in allowed) -> BN -> act."""

    def __init__(self, in_channels, out_channels, kernel_size: IntOrPair, stride=1, dilation=1,
                 act_type="relu", **kwargs):
        conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride,
                         _same_padding(kernel_size, dilation), dilation=dilation,
                         groups=in_channels, bias=False)
        super().__init__(conv, nn.BatchNorm2d(out_channels), Activation(act_type, **kwargs))


class PWConvBNAct(_FusedTail, nn.Sequential):
    """1x1 conv (bias by default) -> BN -> act."""

    def __init__(self, in_channels, out_channels, act_type="relu", bias=True, **kwargs):
        super().__init__(nn.Conv2d(in_channels, out_channels, 1, bias=bias),
                         nn.BatchNorm2d(out_channels), Activation(act_type, **kwargs))


class DSConvBNAct(nn.Sequential):
    """Depth-wise separable: DWConvBNAct (children ``0``) + PWConvBNAct (``1``)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, dilation=1,
                 act_type="relu", **kwargs):
        super().__init__(
            DWConvBNAct(in_channels, in_channels, kernel_size, stride, dilation, act_type, **kwargs),
            PWConvBNAct(in_channels, out_channels, act_type, **kwargs))


class DeConvBNAct(nn.Module):
    """Exact x`scale_factor` transposed-conv upsample -> BN -> act (``up_conv.{0,1,2}``)."""

    def __init__(self, in_channels, out_channels, scale_factor=2, kernel_size=None, padding=None,
                 act_type="relu", **kwargs):
        super().__init__()
        k = 2 * scale_factor - 1 if kernel_size is None else kernel_size
        p = (k - 1) // 2 if padding is None else padding
        self.up_conv = _FusedSequential(
            nn.ConvTranspose2d(in_channels, out_channels, kernel_size=k, stride=scale_factor,
                               padding=p, output_padding=scale_factor - 1),
            nn.BatchNorm2d(out_channels),
            Activation(act_type, **kwargs))

    def forward(self, x):
        return self.up_conv(x)


class _FusedSequential(_FusedTail, nn.Sequential):
    pass


class PyramidPoolingModule(nn.Module):
    """PSP pooling: 4 adaptive-average branches (1x1 conv, C/4) resized back and concatenated."""

    def __init__(self, in_channels, out_channels, act_type, pool_sizes=(1, 2, 4, 6), bias=False):
        super().__init__()
        if len(pool_sizes) != 4:
            raise AssertionError("Length of pool size should be 4.\n")
        hid = in_channels // 4
        for i, ps in enumerate(pool_sizes, start=1):
            setattr(self, f"stage{i}", nn.Sequential(nn.AdaptiveAvgPool2d(ps), conv1x1(in_channels, hid)))
        self.conv = PWConvBNAct(2 * in_channels, out_channels, act_type=act_type, bias=bias)

    def forward(self, x):
        # conv1x1(cat([x, up(s1), .., up(s4)])) == W_x x + sum_i up(W_i s_i): a 1x1 conv commutes
        # with the bilinear resize, so the four full-size branches and their concat (the
        # reference's torch.cat, modules.py:134-158) are never materialised -- each branch's slice
        # of the fuse weight runs on its pooled map (1x1 .. 6x6) and is resized straight into
        # the sum (interpolate's fused skip-add)
        hw, c = x.shape[2:], x.shape[1]
        conv, bn, act = self.conv[0], self.conv[1], self.conv[2]
        y = F.conv2d(x, conv.weight[:, :c], conv.bias)
        for i in range(1, 5):
            s = getattr(self, f"stage{i}")(x)
            lo = c + (i - 1) * s.shape[1]
            y = ops.interpolate(F.conv2d(s, conv.weight[:, lo:lo + s.shape[1]]), hw, True, skip=y)
        return ops.bn_act(y, bn, act, act_module=act)


class SegHead(nn.Sequential):
    """3x3 ConvBNAct (-> hid) + 1x1 classifier."""

    def __init__(self, in_channels, num_class, act_type, hid_channels=128):
        super().__init__(ConvBNAct(in_channels, hid_channels, 3, act_type=act_type),
                         conv1x1(hid_channels, num_class))


def _sync_group(bn):
    """The process group a SyncBatchNorm synchronises over (None: local statistics)."""
    if not isinstance(bn, nn.SyncBatchNorm):
        return None
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return None
    pg = bn.process_group or dist.group.WORLD
    return pg if dist.get_world_size(pg) > 1 else None


def pooled_conv_bn_act(block: nn.Sequential, pooled: torch.Tensor, spatial: int) -> torch.Tensor:
    """``block`` (Sequential conv1x1, BN, act) applied to ``pooled`` [N, C, 1, 1]
    *as if* it had been broadcast to ``spatial`` = H*W positions first.

    The reference attention modules (bisenetv1.py:76-88 ARM, stdc.py via ARM,
    canet/regseg SE variants) do ``pool(x).expand_as(x)`` and then run a 1x1
    conv + BatchNorm over the full H x W map.  Every position holds the same
    vector, so conv and BN batch statistics equal those of the N pooled
    vectors; only BN's *unbiased* running-variance factor uses the expanded
    count N*H*W.  This evaluates the block on the N vectors (H*W times less
    work) with that exact factor, and returns [N, C, 1, 1] for a broadcast
    multiply -- forward values and gradients identical to the reference.
    """
    conv, bn, act = block[0], block[1], block[2]
    y = conv(pooled)
    out_dtype = y.dtype
    if bn.training or not bn.track_running_stats or bn.running_mean is None:
        y32 = y.float()
        pg = _sync_group(bn)
        if pg is None:
            mean = y32.mean(dim=(0, 2, 3))
            var = y32.var(dim=(0, 2, 3), unbiased=False)
            n_vec = y.shape[0]
        else:
            # SyncBatchNorm (reference utils/parallel.py:36-37 converts these too): the batch
            # statistics are over every rank's pooled vectors -- one differentiable all-reduce of
            # (sum, sum of squares, count) in fp64; its backward all-reduces the gradients, as
            # torch's SyncBatchNorm backward does
            from torch.distributed.nn.functional import all_reduce

            y64 = y32.double()
            c = y.shape[1]
            packed = torch.cat([y64.sum(dim=(0, 2, 3)), (y64 * y64).sum(dim=(0, 2, 3)),
                                y64.new_full((1,), float(y.shape[0] * y.shape[2] * y.shape[3]))])
            packed = all_reduce(packed, group=pg)
            tot = packed[2 * c]
            mean64 = packed[:c] / tot
            var = (packed[c:2 * c] / tot - mean64 * mean64).clamp_min(0.0).float()
            mean = mean64.float()
            n_vec = tot.detach().float()  # a device scalar: no host sync
        if bn.training and bn.track_running_stats and bn.running_mean is not None:
            with torch.no_grad():
                count = n_vec * spatial
                mom = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked + 1)
                bn.running_mean.mul_(1 - mom).add_(mean.detach(), alpha=mom)
                unbias = (count / (count - 1).clamp_min(1) if isinstance(count, torch.Tensor)
                          else count / max(count - 1, 1))
                bn.running_var.mul_(1 - mom).add_(var.detach() * unbias, alpha=mom)
                bn.num_batches_tracked.add_(1)
        inv = torch.rsqrt(var + bn.eps)
        y = (y32 - mean[None, :, None, None]) * inv[None, :, None, None]
        if bn.affine:
            y = y * bn.weight[None, :, None, None] + bn.bias[None, :, None, None]
    else:
        y = bn(y)
    return act(y).to(out_dtype)
