"""Depth-wise convolution on the HIP kernels of ``csrc/kernels/dwconv.hip``.

Reference: every ``nn.Conv2d(groups=in_channels)`` of the zoo --
``DWConvBNAct`` (models/modules.py:46-59, incl. BiSeNetV2's x6 channel
multiplier), the raw depth-wise convs of CGNet / MiniNet / DABNet / FDDWNet,
asymmetric (k,1)/(1,k) and dilated (up to 17) variants.  MIOpen has
no fast channels-last depth-wise path, so these run as three hand-written
kernels (forward, gather-form data gradient, two-stage deterministic weight
gradient) on NHWC activations with fp32 accumulation and fp32 weights.

``DepthwiseConv2d`` is an ``nn.Conv2d`` (same parameters and state-dict keys)
whose forward takes the HIP path for channels-last GPU inputs;
:func:`convert_depthwise` swaps the class of every eligible conv of a model in
place.  Under autocast the input is cast to the autocast dtype like
``F.conv2d`` would, while the kernels read the fp32 master weights directly.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .bn import channel_sum
from .dilated import pruned_conv2d
from ._ext import ops, use_hip, write_generation

_DTYPES = (torch.float32, torch.bfloat16, torch.float16)


def _cl_aligned(t: torch.Tensor) -> torch.Tensor:
    if not t.is_contiguous(memory_format=torch.channels_last):
        t = t.contiguous(memory_format=torch.channels_last)
    if t.data_ptr() % 16:
        t = t.clone(memory_format=torch.channels_last)
    return t


def _channels_inner(x: torch.Tensor) -> bool:
    """Channels-last, or a channel slice of a channels-last tensor (FPENet's ``h[:, a:b]`` branch
    inputs, reference models/fpenet.py:78-84): the kernels take the slice as one dense copy
    rather than MIOpen's grouped-conv path (~120 ms per weight gradient at FPENet's shapes)."""
    return x.is_contiguous(memory_format=torch.channels_last) or (x.stride(1) == 1 and x.stride(2) == x.stride(3) * x.shape[3])


def _dw_weight(weight: torch.Tensor, cout: int, taps: int) -> torch.Tensor:
    """fp32 [taps, Cout] weight the kernels read, cached on the parameter while its storage,
    version and the raw-pointer write generation (fused optimizer, BN finalize) are unchanged:
    an inference forward (bf16 weights in the HIP-graph engine) no longer casts and transposes
    every depth-wise weight per call (126 cast + 126 copy kernels per DFANet forward,
    tools/probe_casts.py)."""
    key = (weight.data_ptr(), weight._version, write_generation(), weight.dtype)
    hit = getattr(weight, "_rtseg_dw_wt", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    wt = weight.detach().float().reshape(cout, taps).t().contiguous()
    try:
        weight._rtseg_dw_wt = (key, wt)
    except (AttributeError, RuntimeError):  # a non-leaf view cannot carry attributes
        pass
    return wt


class _DWConvFn(torch.autograd.Function):
    """y = depth-wise conv(x); with ``stats`` also the BN-statistics slab of y (fp32 [rows, 2C],
    produced in the forward kernel's epilogue; ``ops.bn_act(..., part=slab)`` consumes it)."""

    @staticmethod
    def forward(ctx, x, weight, bias, geom, stats=False):
        cout, kh, kw, sh, sw, ph, pw, dh, dw = geom
        wt = _dw_weight(weight, cout, kh * kw)
        b = bias.detach().float().contiguous() if bias is not None else None
        x = _cl_aligned(x)
        part = None
        if stats and b is None:
            y, part = ops().dw_conv_fwd_stats(x, wt, cout, kh, kw, sh, sw, ph, pw, dh, dw)
            if part.numel() == 0:
                part = None
        else:
            y = ops().dw_conv_fwd(x, wt, b, cout, kh, kw, sh, sw, ph, pw, dh, dw)
        ctx.geom = geom
        ctx.has_bias = bias is not None
        ctx.wdtype = weight.dtype
        ctx.wparam = weight  # its strides: DDP's gradient bucket views want them (like_param)
        ctx.save_for_backward(x, wt)
        if not stats:
            return y
        if part is not None:
            ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics slab
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart=None):
        if dy is None:
            return None, None, None, None, None
        x, wt = ctx.saved_tensors
        cout, kh, kw, sh, sw, ph, pw, dh, dw = ctx.geom
        dy = _cl_aligned(dy.to(x.dtype))
        dx = dwt = db = None
        if ctx.needs_input_grad[0]:
            dx = ops().dw_conv_dgrad(dy, wt, x.shape[1], x.shape[2], x.shape[3], kh, kw, sh, sw, ph, pw, dh, dw)
        if ctx.needs_input_grad[1]:
            from .conv import like_param

            dwt = like_param(ops().dw_conv_wgrad(dy, x, kh, kw, sh, sw, ph, pw, dh, dw).to(ctx.wdtype), ctx.wparam)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = channel_sum(dy)
        return dx, dwt, db, None, None


def depthwise_ok(conv: nn.Conv2d) -> bool:
    return (isinstance(conv, nn.Conv2d) and conv.groups > 1 and conv.groups == conv.in_channels
            and conv.out_channels % conv.in_channels == 0 and conv.padding_mode == "zeros"
            and not isinstance(conv.padding, str))


def dw_conv2d(x: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
    """``conv(x)`` for a depth-wise ``conv``; HIP kernels for channels-last GPU inputs
    (``RTSEG_DWCONV=0`` keeps MIOpen, for A/B comparisons)."""
    if x.dim() == 4 and use_hip(x, "dw") and _channels_inner(x) and os.environ.get("RTSEG_DWCONV", "1") != "0":
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        if dt in _DTYPES and conv.weight.dtype in _DTYPES:
            kh, kw = conv.kernel_size
            geom = (conv.out_channels, kh, kw, conv.stride[0], conv.stride[1], conv.padding[0],
                    conv.padding[1], conv.dilation[0], conv.dilation[1])
            return _DWConvFn.apply(x.to(dt), conv.weight, conv.bias, geom)
    # stock fallback (CPU, RTSEG_DISABLE_HIP / RTSEG_HIP_OFF=dw): dead taps dropped first, so a
    # dilated depth-wise conv never reaches the vendor library with padding-only taps
    return pruned_conv2d(x, conv.weight, conv.bias, conv.stride, conv.padding, conv.dilation, conv.groups)


def dw_conv_bn_stats(x: torch.Tensor, conv: nn.Conv2d):
    """Training forward of a depth-wise conv followed by a batch-statistics BN: (y, slab | None),
    the slab holding the BN statistics of y from the conv kernel's epilogue; None -> the caller's
    stock path (``conv(x)`` + ``ops.bn_act``)."""
    if not (x.dim() == 4 and use_hip(x, "dw") and _channels_inner(x)
            and os.environ.get("RTSEG_DWCONV", "1") != "0" and conv.bias is None and depthwise_ok(conv)):
        return None
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
    if dt not in _DTYPES or conv.weight.dtype not in _DTYPES:
        return None
    kh, kw = conv.kernel_size
    geom = (conv.out_channels, kh, kw, conv.stride[0], conv.stride[1], conv.padding[0],
            conv.padding[1], conv.dilation[0], conv.dilation[1])
    return _DWConvFn.apply(x.to(dt), conv.weight, None, geom, True)


DW_BN_FOLDED = [0]  # inference depth-wise conv + eval BN (+ ReLU / ReLU6) passes run as one (tests)


def dw_conv_bn_eval(x: torch.Tensor, conv: nn.Conv2d, bn: nn.Module, act_code: int):
    """Inference ``act(bn_running(dwconv(x)))`` as ONE depth-wise kernel: a depth-wise conv has one
    weight column per output channel, so the eval BN folds exactly into fp32 weights (x scale) and a
    bias (shift + bias x scale), and the ReLU / ReLU6 runs in the store.  BiSeNetV2's gather-expansion
    layers are DW -> BN pairs throughout (reference models/bisenetv2.py).  The folded tensors are
    cached on the conv, keyed on every source's storage / version.  None -> the caller's path."""
    if act_code not in (0, 1, 2) or torch.is_grad_enabled() or not depthwise_ok(conv):
        return None
    if bn.training or not bn.track_running_stats or bn.running_mean is None:
        return None
    if not (x.dim() == 4 and use_hip(x, "dw") and _channels_inner(x) and os.environ.get("RTSEG_DWCONV", "1") != "0"):
        return None
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
    if dt not in _DTYPES or conv.weight.dtype not in _DTYPES:
        return None
    from .bn import eval_coeffs

    kh, kw = conv.kernel_size
    cout = conv.out_channels
    srcs = (conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var)
    key = tuple((t.data_ptr(), t._version) if t is not None else None for t in srcs) + (write_generation(),)
    hit = getattr(conv, "_rtseg_dw_bn", None)
    if hit is None or hit[0] != key:
        _, ss = eval_coeffs(bn)
        scale, shift = ss[:cout], ss[cout:]
        wt = _dw_weight(conv.weight, cout, kh * kw) * scale.view(1, -1)
        b = shift + (conv.bias.detach().float() * scale if conv.bias is not None else 0.0)
        hit = (key, wt.contiguous(), b.contiguous())
        conv._rtseg_dw_bn = hit
    DW_BN_FOLDED[0] += 1
    return ops().dw_conv_fwd(_cl_aligned(x.to(dt)), hit[1], hit[2], cout, kh, kw, conv.stride[0], conv.stride[1],
                             conv.padding[0], conv.padding[1], conv.dilation[0], conv.dilation[1], act_code)


def dw_conv2d_reference(x, weight, bias, stride, padding, dilation):
    return F.conv2d(x, weight, bias, stride, padding, dilation, x.shape[1])


class DepthwiseConv2d(nn.Conv2d):
    """``nn.Conv2d(groups=in_channels)`` routed through the HIP depth-wise kernels."""

    def forward(self, x):
        return dw_conv2d(x, self)


def convert_depthwise(model: nn.Module) -> nn.Module:
    """Swap the class of every eligible depth-wise ``nn.Conv2d`` to :class:`DepthwiseConv2d`
    (in place; parameters and checkpoint keys unchanged)."""
    for m in model.modules():
        if type(m) is nn.Conv2d and depthwise_ok(m):
            m.__class__ = DepthwiseConv2d
    return model
