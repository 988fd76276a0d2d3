"""Transposed convolution on the MFMA implicit-GEMM kernels (K4).

Reference sites: ``DeConvBNAct`` (models/modules.py:89-108, used by 11 models: ADSCNet, CANet,
ERFNet, ESNet, ESPNet, FDDWNet, FSSNet, LinkNet, MiniNet(v2), ShelfNet, SQNet), ENet's
upsampling bottleneck (enet.py:195-197) and AGLNet's GAUM (aglnet.py:134) -- all
``nn.ConvTranspose2d`` on cuDNN in the reference.

A transposed conv with weight W [Cin_t, Cout_t, k, k] IS the input gradient of the conv
``Conv2d(Cout_t -> Cin_t, W)``, so the three passes map onto the conv family of
``conv_igemm.hip`` without col2im, scatter or zero-fill:

* forward  = ``conv_igemm_dgrad`` over x (sub-pixel phases: one launch per output phase, each
  a dense stride-1 gather conv with the taps that reach it) + the bias in the epilogue;
* d input  = ``conv_igemm`` (the ordinary strided forward conv of dy);
* d weight = ``conv_igemm_wgrad`` with (x, dy) in swapped roles; d bias = channel sum of dy.

Each pass needs its reduction channels % 64 == 0 (forward: Cin_t; backward: Cout_t) and the
other side % 8; otherwise that pass runs ``aten.convolution_backward`` / cuDNN-equivalent
MIOpen.  :func:`convert_transposed_convs` swaps the class of every ``nn.ConvTranspose2d``
(parameters / checkpoint keys unchanged).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .bn import channel_sum
from ._ext import ops, use_hip
from .conv import like_param


def _out_size(x, m):
    h, w = x.shape[2:]
    (kh, kw), (sh, sw), (ph, pw) = m.kernel_size, m.stride, m.padding
    (oh, ow), (dh, dw) = m.output_padding, m.dilation
    return ((h - 1) * sh - 2 * ph + dh * (kh - 1) + oh + 1, (w - 1) * sw - 2 * pw + dw * (kw - 1) + ow + 1)


def deconv_ok(x: torch.Tensor, m: nn.Module) -> bool:
    """Forward on our kernel: bf16 channels-last, groups 1, Cin_t % 64, Cout_t % 8."""
    if not isinstance(m, nn.ConvTranspose2d) or m.groups != 1 or m.padding_mode != "zeros":
        return False
    if not x.is_cuda or x.dim() != 4 or not use_hip(x, "deconv"):
        return False
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
    if dt != torch.bfloat16 or m.kernel_size[0] * m.kernel_size[1] > 49:
        return False
    return m.in_channels % 64 == 0 and m.out_channels % 8 == 0


class _DeconvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, m):
        n = x.shape[0]
        ho, wo = _out_size(x, m)
        w16 = weight.detach().to(torch.bfloat16)
        wt = w16.permute(1, 2, 3, 0).contiguous()  # [Cout_t][kh][kw][Cin_t]
        b = bias.detach().float().contiguous() if bias is not None else None
        y = ops().conv_igemm_dgrad(x, wt, [n, m.out_channels, ho, wo], list(m.stride), list(m.padding),
                                   list(m.dilation), b)
        ctx.save_for_backward(x, w16)
        ctx.m = m
        ctx.has_bias = bias is not None
        ctx.wdtype = weight.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w16 = ctx.saved_tensors
        m = ctx.m
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if dy.data_ptr() % 16:
            dy = dy.clone(memory_format=torch.channels_last)
        cin_t, cout_t = m.in_channels, m.out_channels
        st, pd, dl = list(m.stride), list(m.padding), list(m.dilation)
        kh, kw = m.kernel_size
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if cout_t % 64 == 0 and cin_t % 8 == 0:
                wk = w16.permute(0, 2, 3, 1).contiguous()  # [Cin_t][kh][kw][Cout_t]: conv Cout_t -> Cin_t
                dx, _ = ops().conv_igemm(dy, wk, st, pd, dl, False, None, None, 0)
            else:
                dx = torch.ops.aten.convolution_backward(
                    dy, x, w16, None, st, pd, dl, True, list(m.output_padding), 1, [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            w = m.weight
            cl = w.is_contiguous(memory_format=torch.channels_last) and not w.is_contiguous()
            if cout_t % 64 == 0 and cin_t % 64 == 0:
                # [Cin_t][Cout_t][kh][kw], in the parameter's memory order
                dw = ops().conv_igemm_wgrad(dy, x, kh, kw, st, pd, dl, cl or (kh == 1 and kw == 1))
            else:
                dw = torch.ops.aten.convolution_backward(
                    dy, x, w16, None, st, pd, dl, True, list(m.output_padding), 1, [False, True, False])[1]
            dw = like_param(dw.to(ctx.wdtype), w)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = channel_sum(dy)
        return dx, dw, db, None


class _BiasAddFn(torch.autograd.Function):
    """y + bias[c] with the bias gradient through :func:`channel_sum` (see the caller)."""

    @staticmethod
    def forward(ctx, y, bias):
        return y + bias.to(y.dtype).view(1, -1, 1, 1)

    @staticmethod
    def backward(ctx, g):
        gb = channel_sum(g) if ctx.needs_input_grad[1] else None
        return g, gb


def conv_transpose2d(x: torch.Tensor, m: nn.ConvTranspose2d, output_size=None) -> torch.Tensor:
    if deconv_ok(x, m) and output_size is None:
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if x.data_ptr() % 16:
            x = x.clone(memory_format=torch.channels_last)
        return _DeconvFn.apply(x, m.weight, m.bias, m)
    if (m.bias is not None and m.bias.requires_grad and torch.is_grad_enabled() and x.is_cuda and use_hip(x, "deconv")
            and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)):
        # Shapes our kernel does not take (e.g. the x8 19 -> 19 class heads of CANet / ADSCNet at
        # full resolution): MIOpen without the bias, the bias added separately -- aten's own bias
        # gradient for a channels-last [8, 19, 1024, 2048] output took 63 ms (profiles/r3_models)
        op = m._output_padding(x, output_size, list(m.stride), list(m.padding), list(m.kernel_size), 2,
                               list(m.dilation))
        y = F.conv_transpose2d(x, m.weight, None, m.stride, m.padding, op, m.groups, m.dilation)
        return _BiasAddFn.apply(y, m.bias)
    return nn.ConvTranspose2d.forward(m, x, output_size)


class TransposedConv2d(nn.ConvTranspose2d):
    """``nn.ConvTranspose2d`` whose GPU bf16 forward / backward run on the MFMA kernels."""

    def forward(self, x, output_size=None):
        return conv_transpose2d(x, self, output_size)


def convert_transposed_convs(model: nn.Module) -> nn.Module:
    for mod in model.modules():
        if type(mod) is nn.ConvTranspose2d:
            mod.__class__ = TransposedConv2d
    return model


def deconv_reference(x, weight, bias, stride, padding, output_padding, dilation):
    return F.conv_transpose2d(x, weight, bias, stride, padding, output_padding, 1, dilation)
