"""Narrow dilated 1-D convolutions as a sum of per-tap GEMMs.

Reference: CFPNet's ``FeaturePyramidChannel`` (reference models/cfpnet.py:108-138) stacks
dense ``(3, 1)`` / ``(1, 3)`` ConvBNActs with dilation up to 16 on 4..16 channels.  On
MI355X, MIOpen's solver search for these shapes in channels-last at 1024x512 faulted the
GPU (illegal memory access inside ``EvaluateInvokers``; tools/zoo_fps.py run of this round),
so such layers do not go through MIOpen at all.  A K-tap 1-D conv with C_in, C_out <= 16
is a bandwidth-bound op, and in NHWC it is exactly

    y[n, h, w, :] = sum_t  x[n, h + (t - (K-1)/2) * d, w, :] @ W_t        (zero outside)

On the GPU the forward and the data gradient run on ``csrc/kernels/tapconv.hip`` (one
thread per pixel, weights in LDS, one read of x / one write of y; the data gradient is the
same kernel with flipped taps and transposed W_t); the weight gradient is K small GEMMs
over shifted views of one zero-padded copy of ``x`` -- the formulation :func:`tap_conv2d`
also uses for CPU tensors (autograd, identical numerics up to summation order).
:func:`convert_tap_convs` swaps the class of every eligible ``nn.Conv2d`` (parameters and
checkpoint keys unchanged).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .bn import channel_sum
from .dilated import pruned_conv2d
from ._ext import ops, use_hip

MAX_CHANNELS = 16
HIP_CHANNELS = (4, 8, 16)


def tapconv_ok(conv: nn.Module) -> bool:
    if not isinstance(conv, nn.Conv2d) or conv.groups != 1 or conv.padding_mode != "zeros":
        return False
    if isinstance(conv.padding, str) or tuple(conv.stride) != (1, 1):
        return False
    kh, kw = conv.kernel_size
    if min(kh, kw) != 1 or max(kh, kw) < 2 or max(kh, kw) % 2 == 0:
        return False
    axis = 0 if kh > 1 else 1
    d, p = conv.dilation[axis], conv.padding[axis]
    if d < 2 or p != d * (max(kh, kw) - 1) // 2 or conv.padding[1 - axis] != 0:
        return False
    return conv.in_channels <= MAX_CHANNELS and conv.out_channels <= MAX_CHANNELS


def tap_conv2d(x: torch.Tensor, weight: torch.Tensor, bias, dilation: int, axis: int) -> torch.Tensor:
    """Same-padded stride-1 1-D conv along H (axis 0) or W (axis 1) of ``x`` [N, C, H, W]."""
    k = weight.shape[2 + axis]
    p = dilation * (k - 1) // 2
    xn = x.permute(0, 2, 3, 1)                                  # NHWC view (free for channels-last)
    pad = (0, 0, 0, 0, p, p) if axis == 0 else (0, 0, p, p)
    xp = F.pad(xn, pad)
    n = x.shape[2 + axis]
    w = weight.squeeze(3 - axis)                                # [Cout, Cin, K]
    y = None
    for t in range(k):
        sl = xp.narrow(1 + axis, t * dilation, n)
        term = torch.matmul(sl, w[:, :, t].t())
        y = term if y is None else y + term
    if bias is not None:
        y = y + bias
    return y.permute(0, 3, 1, 2)                                # NCHW logical, channels-last memory


def _outer_sum(a, b, chunk=8192):
    """a^T b for a [M, P], b [M, Q] with M in the millions and P, Q <= 16: a batched product over
    M-chunks, then a sum over the chunks.  As one GEMM with K = M (round 2) hipBLASLt ran it on a
    handful of 16 x 16 output tiles: 290 us per call, 70 ms per CFPNet training step."""
    m = a.shape[0]
    nb = m // chunk
    out = None
    if nb > 0:
        out = torch.bmm(a[: nb * chunk].view(nb, chunk, -1).transpose(1, 2), b[: nb * chunk].view(nb, chunk, -1)).sum(0)
    if nb * chunk < m:
        r = a[nb * chunk:].t() @ b[nb * chunk:]
        out = r if out is None else out + r
    return out


def _shift_wgrad(x, gy, k, dilation, axis):
    """dW [Cout, Cin, K] = sum_p gy_p^T shift_t(x)_p over one padded copy of x (fp32 accumulation)."""
    p = dilation * (k - 1) // 2
    xn = x.permute(0, 2, 3, 1)
    xp = F.pad(xn, (0, 0, 0, 0, p, p) if axis == 0 else (0, 0, p, p))
    n = x.shape[2 + axis]
    g2 = gy.permute(0, 2, 3, 1).reshape(-1, gy.shape[1]).float().contiguous()
    cols = [_outer_sum(g2, xp.narrow(1 + axis, t * dilation, n).reshape(-1, x.shape[1]).float().contiguous())
            for t in range(k)]
    return torch.stack(cols, dim=2)


class _TapConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, dilation, axis):
        k = weight.shape[2 + axis]
        w = weight.detach().float().squeeze(3 - axis)                 # [Cout, Cin, K]
        wf = w.permute(2, 1, 0).contiguous()                          # [K, Cin, Cout]
        b = bias.detach().float().contiguous() if bias is not None else x.new_empty(0, dtype=torch.float32)
        y = ops().tapconv_fwd(x, wf, b, dilation, axis)
        ctx.save_for_backward(x, weight)
        ctx.geo = (k, dilation, axis, bias is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        k, dilation, axis, has_b = ctx.geo
        gy = gy.contiguous(memory_format=torch.channels_last)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            w = weight.detach().float().squeeze(3 - axis)             # [Cout, Cin, K]
            wb = w.flip(2).permute(2, 0, 1).contiguous()              # [K, Cout, Cin], taps flipped
            gx = ops().tapconv_fwd(gy, wb, gy.new_empty(0, dtype=torch.float32), dilation, axis)
        if ctx.needs_input_grad[1]:
            gw = _shift_wgrad(x, gy, k, dilation, axis).unsqueeze(3 - axis).to(weight.dtype)
        if has_b and ctx.needs_input_grad[2]:
            gb = channel_sum(gy).to(weight.dtype)
        return gx, gw, gb, None, None


def hip_tapconv_ok(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (use_hip(x, "tapconv") and conv.in_channels in HIP_CHANNELS and conv.out_channels in HIP_CHANNELS
            and max(conv.kernel_size) <= 7 and x.dtype in (torch.float32, torch.bfloat16))


class TapConv2d(nn.Conv2d):
    """``nn.Conv2d`` routed to the tap-conv HIP kernel on the GPU (see module docstring)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            return pruned_conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups)
        axis = 0 if self.kernel_size[0] > 1 else 1
        if torch.is_autocast_enabled("cuda"):
            x = x.to(torch.get_autocast_dtype("cuda"))
        if hip_tapconv_ok(x, self):
            x = x.contiguous(memory_format=torch.channels_last)
            return _TapConvFn.apply(x, self.weight, self.bias, self.dilation[axis], axis)
        return tap_conv2d(x, self.weight, self.bias, self.dilation[axis], axis)


def convert_tap_convs(model: nn.Module) -> nn.Module:
    """Swap the class of every eligible narrow dilated 1-D ``nn.Conv2d`` to :class:`TapConv2d`."""
    for m in model.modules():
        if type(m) is nn.Conv2d and tapconv_ok(m):
            m.__class__ = TapConv2d
    return model
