"""Dense convolution on the MFMA implicit-GEMM kernel (``csrc/kernels/conv_mfma.hip``).

Reference: the ``nn.Conv2d`` of every ConvBNAct / residual block (models/modules.py:73-85,
ddrnet.py:168-219), executed by cuDNN in the reference and followed by a separate
BatchNorm pass.  Here, for channels-last bf16 activations:

* training: ``conv_bn_stats`` runs the conv with the BN statistics in its epilogue
  (per-channel sum / sum of squares -> a [G, 2C] slab that ``ops.bn_act`` finalizes),
  so the BatchNorm forward no longer re-reads the conv output; the backward is
  ``aten.convolution_backward`` (MIOpen dgrad / wgrad);
* inference: ``conv_bn_act_eval`` folds BatchNorm (running statistics), the residual
  add and ReLU / ReLU6 into the conv epilogue -- one kernel per ConvBNAct / RB tail.

Whether a layer takes this path or MIOpen (+ the separate BN pass) is decided per
shape by timing both the first time the shape is seen (``cudnn.benchmark``-style,
outside graph capture); ``RTSEG_CONV_MFMA=0`` disables the path, ``=1`` forces it.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import ops, use_hip

_DECISIONS: dict = {}


def _mode() -> str:
    return os.environ.get("RTSEG_CONV_MFMA", "auto")


def conv_ok(x: torch.Tensor, conv: nn.Module) -> bool:
    """Shapes/layouts the kernel handles (anything else stays on MIOpen)."""
    if type(conv) is not nn.Conv2d or conv.groups != 1 or conv.bias is not None:
        return False
    if conv.padding_mode != "zeros" or isinstance(conv.padding, str):
        return False
    if x.dim() != 4 or not x.is_cuda or conv.in_channels % 32 or conv.out_channels % 8:
        return False
    if _mode() == "0" or not use_hip(x):
        return False
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
    if dt != torch.bfloat16:
        return False
    return x.is_contiguous(memory_format=torch.channels_last)


def _geom(conv):
    return list(conv.stride), list(conv.padding), list(conv.dilation)


def weight_krsc(conv: nn.Conv2d) -> torch.Tensor:
    """bf16 [Cout, KH, KW, Cin] copy of the weight, cached until the parameter changes."""
    w = conv.weight
    key = (w.data_ptr(), w._version, w.dtype)
    cached = getattr(conv, "_rtseg_wk", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    wk = w.detach().to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
    if not torch.is_grad_enabled() or not conv.training:
        conv._rtseg_wk = (key, wk)  # eval / inference: weights are static between steps
    return wk


class _ConvStatsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, wk, stride, padding, dilation):
        y, part = ops().conv_mfma(x, wk, stride, padding, dilation, True, None, None, 0)
        ctx.save_for_backward(x, wk)
        ctx.geom = (stride, padding, dilation)
        ctx.wdtype = weight.dtype
        ctx.mark_non_differentiable(part)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart):
        x, wk = ctx.saved_tensors
        stride, padding, dilation = ctx.geom
        w4 = wk.permute(0, 3, 1, 2)  # [Cout, Cin, KH, KW] with channels-last strides
        dy = dy.contiguous(memory_format=torch.channels_last)
        mask = [ctx.needs_input_grad[0], ctx.needs_input_grad[1], False]
        dx, dw, _ = torch.ops.aten.convolution_backward(dy, x, w4, None, stride, padding, dilation, False,
                                                         [0, 0], 1, mask)
        if dw is not None:
            dw = dw.to(ctx.wdtype)
        return dx, dw, None, None, None, None


def _time(fn, reps=10):
    """GPU time of ``fn``: captured into a HIP graph and replayed, so two candidates with
    different launch counts are compared the way a captured / GPU-bound step runs them
    (eager timing of ~20 us kernels measures the host launch path instead)."""
    fn()  # warm-up: MIOpen find / kernel load happen outside the capture
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        g.replay()
        s.record()
        for _ in range(reps):
            g.replay()
        e.record()
    except RuntimeError:  # capture not possible here: fall back to eager timing
        s.record()
        for _ in range(reps):
            fn()
        e.record()
    e.synchronize()
    return s.elapsed_time(e)


def _decide(key, ours, theirs) -> bool:
    """True -> MFMA path.  Timed once per key (never while a HIP graph is being captured)."""
    mode = _mode()
    if mode == "1":
        return True
    got = _DECISIONS.get(key)
    if got is not None:
        return got
    if torch.cuda.is_current_stream_capturing():
        return False
    with torch.no_grad():
        t_ours, t_theirs = _time(ours), _time(theirs)
    _DECISIONS[key] = t_ours < t_theirs
    return _DECISIONS[key]


def conv_bn_stats(x: torch.Tensor, conv: nn.Conv2d):
    """Training forward: (y, slab) with the BN statistics of y, or None -> caller uses MIOpen."""
    x = x.to(torch.bfloat16)
    stride, padding, dilation = _geom(conv)
    wk = weight_krsc(conv)
    key = ("train", tuple(x.shape), conv.out_channels, conv.kernel_size, tuple(stride), tuple(padding),
           tuple(dilation))

    def ours():
        ops().conv_mfma(x, wk, stride, padding, dilation, True, None, None, 0)

    def theirs():
        ops().bn_stats_sums(F.conv2d(x, wk.permute(0, 3, 1, 2), None, stride, padding, dilation))

    if not _decide(key, ours, theirs):
        return None
    return _ConvStatsFn.apply(x, conv.weight, wk, stride, padding, dilation)


def conv_bn_act_eval(x: torch.Tensor, conv: nn.Conv2d, bn: nn.Module, act_code: int, residual=None):
    """Inference: act(BN_running(conv(x)) + residual) in one kernel, or None -> caller's path."""
    if bn.training or not bn.track_running_stats or bn.running_mean is None or act_code not in (0, 1, 2):
        return None
    if residual is not None and not (residual.is_contiguous(memory_format=torch.channels_last)
                                     and residual.dim() == 4):
        return None
    x = x.to(torch.bfloat16)
    res = residual.to(torch.bfloat16) if residual is not None else None
    stride, padding, dilation = _geom(conv)
    wk = weight_krsc(conv)
    from .bn import eval_coeffs

    _, ss = eval_coeffs(bn)
    key = ("eval", tuple(x.shape), conv.out_channels, conv.kernel_size, tuple(stride), tuple(padding),
           tuple(dilation), res is not None)

    def ours():
        ops().conv_mfma(x, wk, stride, padding, dilation, False, ss, res, act_code)

    def theirs():
        y = F.conv2d(x, wk.permute(0, 3, 1, 2), None, stride, padding, dilation)
        ops().bn_apply(y, ss, res, act_code)

    if not _decide(key, ours, theirs):
        return None
    y, _ = ops().conv_mfma(x, wk, stride, padding, dilation, False, ss, res, act_code)
    return y


def conv_forward(x: torch.Tensor, conv: nn.Module) -> torch.Tensor:
    """``conv(x)``; in bf16-autocast inference the bf16 weight copy is cached on the module
    (autocast would re-cast the fp32 weight -- one extra kernel per conv -- every forward)."""
    if (type(conv) is nn.Conv2d and not conv.training and not torch.is_grad_enabled() and x.is_cuda
            and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        w = conv.weight
        key = (w.data_ptr(), w._version, None if conv.bias is None else (conv.bias.data_ptr(), conv.bias._version))
        hit = getattr(conv, "_rtseg_w16", None)
        if hit is None or hit[0] != key:
            b16 = conv.bias.detach().to(torch.bfloat16) if conv.bias is not None else None
            hit = conv._rtseg_w16 = (key, w.detach().to(torch.bfloat16), b16)
        with torch.autocast("cuda", enabled=False):
            return conv._conv_forward(x.to(torch.bfloat16), hit[1], hit[2])
    return conv(x)


def conv_bn_act(x: torch.Tensor, conv: nn.Module, bn: nn.Module, act="none", residual=None, act_module=None):
    """``act(bn(conv(x)) + residual)`` with the conv on the MFMA kernel when it wins: BN
    statistics in its epilogue (training) or the whole BN + residual + activation tail
    (inference).  Any other case is ``conv`` followed by ``ops.bn_act``."""
    from .bn import act_code, bn_act

    if conv_ok(x, conv) and isinstance(bn, (nn.BatchNorm2d, nn.SyncBatchNorm)):
        code = act if isinstance(act, int) else act_code(act)
        if code is not None:
            use_batch = bn.training or not bn.track_running_stats or bn.running_mean is None
            if not use_batch:
                y = conv_bn_act_eval(x, conv, bn, code, residual)
                if y is not None:
                    return y
            else:
                r = conv_bn_stats(x, conv)
                if r is not None:
                    return bn_act(r[0], bn, code, residual=residual, act_module=act_module, part=r[1])
    return bn_act(conv_forward(x, conv), bn, act, residual=residual, act_module=act_module)


def decisions() -> dict:
    """Per-shape autotune outcomes so far (for logs / profiles)."""
    return dict(_DECISIONS)
