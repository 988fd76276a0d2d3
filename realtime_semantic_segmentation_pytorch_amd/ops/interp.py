"""Bilinear resize with fused ``+ skip`` and activation (HIP kernel ``interp.hip``).

Drop-in for ``F.interpolate(x, size, mode='bilinear', align_corners=...)`` and
for the ubiquitous fusion pattern ``act(skip + F.interpolate(x, size))``
(reference models/ddrnet.py:233-236, ddrnet.py:275-289, modules.py:150-153,
swiftnet.py:60-70, bisenetv2.py:213-218 ...).
"""
from __future__ import annotations

import os
import threading
import weakref
from contextlib import contextmanager
from typing import Optional, Sequence

import torch
import torch.nn.functional as F

from ._ext import use_hip, ops

ACT_CODES = {None: 0, "none": 0, "relu": 1, "relu6": 2}
# skip-gradient hand-off to a sibling routed conv (RTSEG_SKIP_HANDOFF=0: off, for A/B)
_SKIP_HANDOFF = os.environ.get("RTSEG_SKIP_HANDOFF", "1") != "0"
SKIP_HANDOFFS = [0]  # backward passes that handed the skip gradient over (tests)


def _torch_act(y: torch.Tensor, act: int) -> torch.Tensor:
    if act == 1:
        return F.relu(y)
    if act == 2:
        return F.relu6(y)
    return y


def _will_run(node) -> bool:
    """Whether autograd node ``node`` executes in the backward pass now running: it is in the
    current graph task (reachable from the roots) and not pruned by ``inputs=``.  A sibling conv
    whose output was dropped, or feeds only another loss, is NOT -- handing it the skip gradient
    would lose that gradient."""
    try:
        return bool(torch._C._will_engine_execute_node(node))
    except (AttributeError, RuntimeError, TypeError):
        return False


class _InterpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, skip, out_h, out_w, align, act):
        y = ops().interp(x, out_h, out_w, align, skip, act)
        ctx.align = align
        ctx.act = act
        ctx.in_hw = (x.shape[2], x.shape[3])
        ctx.cl = x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous()
        ctx.has_skip = skip is not None
        # a routed conv that also reads the skip tensor (a sibling consumer, e.g. DDRNet's
        # bilateral-fusion 3 x 3 conv on x_high): the skip gradient may go to its dgrad epilogue
        ctx.skip_conv = None
        if skip is not None and _SKIP_HANDOFF and ctx.needs_input_grad[1]:
            from .conv import consumer_for

            node = consumer_for(skip)
            if node is not None:
                ctx.skip_conv = weakref.ref(node)
        if act:
            ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        if ctx.act:
            (y,) = ctx.saved_tensors
            g = ops().act_mask(g, y, ctx.act)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = ops().interp_backward(g, ctx.in_hw[0], ctx.in_hw[1], ctx.align, ctx.cl)
        gs = g if (ctx.has_skip and ctx.needs_input_grad[1]) else None
        if gs is not None and ctx.skip_conv is not None:
            node = ctx.skip_conv()
            if node is not None and not node.ran and node.addend_slot is None and _will_run(node):
                # the conv node has not run and will run in THIS backward (its output reaches the
                # roots): it adds gs in its dgrad epilogue (no accumulation add)
                node.addend_slot = [gs]
                gs = None
                SKIP_HANDOFFS[0] += 1
        return gx, gs, None, None, None, None


def interpolate(x: torch.Tensor, size: Sequence[int], align_corners: bool = True,
                skip: Optional[torch.Tensor] = None, act: Optional[str] = None) -> torch.Tensor:
    """``act(skip + bilinear_resize(x, size))`` in one HIP kernel on GPU."""
    out_h, out_w = int(size[0]), int(size[1])
    code = ACT_CODES[act]
    if use_hip(x, "interp") and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16, torch.float16):
        if skip is not None and skip.dtype != x.dtype:
            dt = torch.promote_types(skip.dtype, x.dtype)
            x, skip = x.to(dt), skip.to(dt)
        return _InterpFn.apply(x, skip, out_h, out_w, bool(align_corners), code)
    y = F.interpolate(x, (out_h, out_w), mode="bilinear", align_corners=align_corners)
    if skip is not None:
        y = y + skip
    return _torch_act(y, code)


# --------------------------------------------------------------------------
# Deferred final upsample: the trainer asks models to hand back their logits at
# head resolution, and the fused loss kernel interpolates inside the loss.
# --------------------------------------------------------------------------
_defer = threading.local()


@contextmanager
def defer_final_upsample(enabled: bool = True):
    prev = getattr(_defer, "on", False)
    _defer.on = enabled
    try:
        yield
    finally:
        _defer.on = prev


class DeferredLogits:
    """Head-resolution logits plus the resize that the model would have applied."""

    __slots__ = ("logits", "size", "align_corners")

    def __init__(self, logits: torch.Tensor, size, align_corners: bool):
        self.logits = logits
        self.size = (int(size[0]), int(size[1]))
        self.align_corners = align_corners

    def materialize(self) -> torch.Tensor:
        if tuple(self.logits.shape[2:]) == self.size:
            return self.logits
        return interpolate(self.logits, self.size, self.align_corners)

    # minimal tensor-like surface used by trainers / metrics
    @property
    def shape(self):
        return torch.Size((self.logits.shape[0], self.logits.shape[1]) + self.size)

    def size_(self):
        return self.shape

    def detach(self):
        return DeferredLogits(self.logits.detach(), self.size, self.align_corners)


try:  # let DDP / torch.compile see through DeferredLogits (DDP walks forward outputs)
    from torch.utils import _pytree as _pt

    _pt.register_pytree_node(
        DeferredLogits,
        lambda d: ([d.logits], (d.size, d.align_corners)),
        lambda ch, ctx: DeferredLogits(ch[0], ctx[0], ctx[1]),
    )
except Exception:  # pragma: no cover - older torch
    pass


def final_upsample(x: torch.Tensor, size, align_corners: bool = True):
    """Model-output resize; returns :class:`DeferredLogits` inside ``defer_final_upsample``."""
    if getattr(_defer, "on", False) and torch.is_grad_enabled():
        return DeferredLogits(x, size, align_corners)
    if tuple(x.shape[2:]) == (int(size[0]), int(size[1])):
        return x
    return interpolate(x, size, align_corners)


def materialize(x):
    return x.materialize() if isinstance(x, DeferredLogits) else x
