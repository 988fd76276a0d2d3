"""Point-wise activation family on the HIP kernels (``csrc/kernels/act.hip``).

Reference: models/modules.py:111-131 (the ``Activation`` hub: PReLU, LeakyReLU, ELU, CELU,
SELU, Hardswish, Hardtanh, SiLU, Sigmoid, Tanh, GELU, ...), used by every ConvBNAct-style block
of the zoo -- PReLU dominates ENet / ESPNet(v2) / CGNet / DABNet / CFPNet / FSSNet.

The backward recomputes f'(x) from the saved input; PReLU's backward writes dx and the
(per-channel or scalar) weight gradient in one deterministic pass, where stock PyTorch runs
an elementwise pass plus a separate reduction.  :func:`convert_activations` swaps the class of
every supported activation module (parameters and state_dict keys unchanged), like
``convert_batchnorm`` / ``convert_pooling``.  CPU tensors (and ``RTSEG_DISABLE_HIP=1``) run the
module's own PyTorch forward.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ._ext import ops, use_hip

(PRELU, LEAKY, ELU, CELU, SELU, HARDSWISH, HARDTANH, SILU, SIGMOID, TANH, GELU, GELU_TANH) = range(12)


def kind_of(m: nn.Module):
    """(kind, a, b, weight) for a supported activation module, else None."""
    if isinstance(m, nn.PReLU):
        return PRELU, 0.0, 0.0, m.weight
    if isinstance(m, nn.LeakyReLU):
        return LEAKY, float(m.negative_slope), 0.0, None
    if isinstance(m, nn.ELU):
        return ELU, float(m.alpha), 0.0, None
    if isinstance(m, nn.CELU):
        return CELU, float(m.alpha), 0.0, None
    if isinstance(m, nn.SELU):
        return SELU, 0.0, 0.0, None
    if isinstance(m, nn.Hardswish):
        return HARDSWISH, 0.0, 0.0, None
    if isinstance(m, nn.Hardtanh):  # ReLU6 included
        return HARDTANH, float(m.min_val), float(m.max_val), None
    if isinstance(m, nn.SiLU):
        return SILU, 0.0, 0.0, None
    if isinstance(m, nn.Sigmoid):
        return SIGMOID, 0.0, 0.0, None
    if isinstance(m, nn.Tanh):
        return TANH, 0.0, 0.0, None
    if isinstance(m, nn.GELU):
        return (GELU_TANH if m.approximate == "tanh" else GELU), 0.0, 0.0, None
    return None


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, kind, a, b):
        ctx.kind, ctx.a, ctx.b = kind, a, b
        ctx.save_for_backward(x, w)
        return ops().act_fwd(x, kind, w, a, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx, dw = ops().act_bwd(dy, x, ctx.kind, w, ctx.a, ctx.b)
        want_w = w is not None and ctx.needs_input_grad[1]
        return dx, (dw if want_w else None), None, None, None


def _ok(x: torch.Tensor, w) -> bool:
    if x.dtype not in (torch.float32, torch.bfloat16, torch.float16) or x.numel() == 0:
        return False
    dense = x.is_contiguous() or (x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last))
    if not dense or x.numel() >= 2 ** 32:
        return False
    if w is not None:
        if w.dtype != torch.float32 or not w.is_cuda:
            return False
        if w.numel() > 1 and (x.dim() < 2 or x.shape[1] != w.numel() or w.numel() > 4096):
            return False
    return use_hip(x, "act")


def activation(x: torch.Tensor, module: nn.Module) -> torch.Tensor:
    """``module(x)`` on the HIP kernels when possible."""
    spec = kind_of(module)
    if spec is not None and x.is_cuda:
        kind, a, b, w = spec
        if _ok(x, w):
            if w is not None:
                w = w.contiguous()
            return _ActFn.apply(x, w, kind, a, b)
    return super(_HipAct, module).forward(x) if isinstance(module, _HipAct) else module(x)


class _HipAct:
    """Mixin: forward on the HIP activation kernels (class-swapped onto torch modules)."""

    def forward(self, x):
        return activation(x, self)


_SWAPPABLE = (nn.PReLU, nn.LeakyReLU, nn.ELU, nn.CELU, nn.SELU, nn.Hardswish, nn.Hardtanh, nn.SiLU,
              nn.Sigmoid, nn.Tanh, nn.GELU)
_HIP_CLASSES = {}


def _hip_class(cls):
    if cls not in _HIP_CLASSES:
        _HIP_CLASSES[cls] = type(f"Hip{cls.__name__}", (_HipAct, cls), {})
    return _HIP_CLASSES[cls]


def convert_activations(model: nn.Module) -> nn.Module:
    """Swap every supported activation module onto the HIP kernels (in place).  ReLU itself
    stays on PyTorch (in-place ``relu_`` is already one pass; the conv / BN epilogues fuse it)."""
    for m in model.modules():
        if type(m) in _SWAPPABLE:
            m.__class__ = _hip_class(type(m))
    return model


__all__ = ["activation", "convert_activations", "kind_of"]
