"""Attention gating (K10): ``x * s``, ``x * (1 + s)`` or ``x * s + y * (1 - s)`` in one pass.

``s`` is the gate (or ``sigmoid(gate)`` when ``sigmoid=True``, computed in-kernel) broadcast
per channel (``[N, C, 1, 1]``: squeeze-excite, ARM, FFM, CGNet, CANet), per pixel
(``[N, 1, H, W]``: PP-LiteSeg's spatial UAFM) or full-size (BiSeNetV2's BGA).

Reference sites: bisenetv1.py:76-114, regseg.py:109-127, cgnet.py:105-108, canet.py:107-117,
pp_liteseg.py:120-141, aglnet.py:95-111, bisenetv2.py:140-162 -- there each gate is 2-4 stock
ops (expand, sigmoid, mul, add), each a full pass over the activation; here one HIP kernel
forward (``gate.hip``) and one backward that also reduces the gate gradient.  Anything the
kernels do not take (CPU, non-channels-last, mixed shapes) runs the same math in PyTorch.
"""
from __future__ import annotations

from typing import Optional

import torch

from ._ext import ops, use_hip

MODES = {"mul": 0, "residual": 1, "blend": 2}
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def gate_reference(x, att, other=None, mode="mul", sigmoid=False):
    s = torch.sigmoid(att) if sigmoid else att
    if mode == "mul":
        return x * s
    if mode == "residual":
        return x + x * s
    return x * s + other * (1 - s)


def _bcast(x, att) -> int:
    n, c, h, w = x.shape
    if att.shape[1] == c and att.shape[2] == 1 and att.shape[3] == 1 and h * w > 1:
        return 0
    if att.shape[1] == 1 and att.shape[2] == h and att.shape[3] == w and c > 1:
        return 1
    return 2 if tuple(att.shape) == tuple(x.shape) else -1


def _cl(t):
    t = t.contiguous(memory_format=torch.channels_last)
    return t if t.data_ptr() % 16 == 0 else t.clone(memory_format=torch.channels_last)


class _GateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, att, other, mode, sigmoid):
        out = ops().gate_fwd(x, att, other, mode, sigmoid)
        ctx.save_for_backward(x, att, other)
        ctx.mode, ctx.sigmoid = mode, sigmoid
        return out

    @staticmethod
    def backward(ctx, go):
        x, att, other = ctx.saved_tensors
        gx, gy, ga = ops().gate_bwd(_cl(go.to(x.dtype)), x, att, other, ctx.mode, ctx.sigmoid)
        return gx, ga, (gy if ctx.mode == 2 else None), None, None


def gate(x: torch.Tensor, att: torch.Tensor, other: Optional[torch.Tensor] = None, mode: str = "mul",
         sigmoid: bool = False) -> torch.Tensor:
    """Gate ``x`` by ``att`` (see module doc); ``other`` is the second input of ``mode='blend'``.
    The result has ``x``'s dtype (a bf16 activation gated by an fp32 gate stays bf16)."""
    code = MODES[mode]
    if (x.is_cuda and use_hip(x, "gate") and x.dim() == 4 and att.dim() == 4 and x.dtype in _DT
            and att.shape[0] == x.shape[0] and x.numel() > 0):
        bc = _bcast(x, att)
        ok = bc >= 0 and (other is None) == (code != 2)
        if ok and other is not None:
            ok = other.shape == x.shape
        if ok and ops().gate_supported(_DT[x.dtype], x.shape[1], bc):
            xx = _cl(x)
            oo = _cl(other.to(x.dtype)) if other is not None else None
            aa = _cl(att.to(x.dtype)) if bc == 2 else att.float().contiguous()
            return _GateFn.apply(xx, aa, oo, code, sigmoid)
    out = gate_reference(x, att, other, mode, sigmoid)
    return out.to(x.dtype) if x.is_floating_point() else out  # output in x's dtype, as the kernel
