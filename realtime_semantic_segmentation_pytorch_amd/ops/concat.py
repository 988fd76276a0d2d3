"""Concat elimination: branch outputs land in ONE channels-last buffer.

Reference sites: STDC's ``torch.cat([x1, x2, x3, x4], dim=1)`` at the end of every
``STDCModule`` (models/stdc.py:104-128) and DDRNet's DAPPM ``torch.cat`` of its five
branches (models/ddrnet.py:241-291).  ``torch.cat`` re-reads every branch and writes
the result; its backward hands each branch a strided slice of the result's gradient,
which the branch's BN backward then copies to a dense tensor (or autograd adds into
the gradient of the branch's other consumer).

Here, with a :class:`ConcatSink`:

* forward: the fused BN(+act) kernel of each branch (``ops.bn_act(..., sink=(s, i))``)
  stores its output twice -- dense, for the branch's own consumers (the next conv), and
  into its channel slice of the sink's buffer (``bn_apply(out2=...)``, 16-byte vectors
  at the buffer's row stride).  :meth:`ConcatSink.cat` then returns the buffer: no cat
  kernel (a branch no kernel wrote, e.g. STDC's pooled ``x1``, is copied in);
* backward: the cat node gives each written branch's BN node its gradient slice -- a
  strided view of the buffer's gradient, never copied -- which the BN backward kernels
  read at its row stride and add to the gradient from the branch's other consumers
  (``bn_backward(grad2=...)``): no slice copy, no gradient-accumulation add.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import torch

# RTSEG_CONCAT_SINK=0: plain torch.cat (A/B runs, tests/test_concat_gpu.py)
_ENABLED = os.environ.get("RTSEG_CONCAT_SINK", "1") != "0"


class ConcatSink:
    """The concat buffer of branches of ``widths`` channels (in concat order)."""

    def __init__(self, widths: Sequence[int]):
        self.widths = [int(w) for w in widths]
        self.offsets = [sum(self.widths[:i]) for i in range(len(self.widths))]
        self.total = sum(self.widths)
        self.buf: Optional[torch.Tensor] = None
        self.written: dict = {}  # branch index -> (output tensor, its BN autograd node)

    def slot(self, i: int, like: torch.Tensor) -> Optional[torch.Tensor]:
        """Channel slice ``i`` of the buffer for a branch output shaped like ``like`` (allocated
        on first use), or None when the fused kernels cannot store there."""
        if like.dim() != 4 or like.shape[1] != self.widths[i] or not like.is_cuda or not _ENABLED:
            return None
        if torch.onnx.is_in_onnx_export() or torch.jit.is_tracing():
            return None  # exported graphs keep the plain cat
        vec = 16 // like.element_size()
        if self.offsets[i] % vec or self.total % vec or self.widths[i] % vec or self.widths[i] // vec > 256:
            return None
        n, _, h, w = like.shape
        if self.buf is None:
            self.buf = torch.empty((n, self.total, h, w), dtype=like.dtype, device=like.device,
                                   memory_format=torch.channels_last)
        elif self.buf.dtype != like.dtype or self.buf.shape[0] != n or tuple(self.buf.shape[2:]) != (h, w):
            return None
        return self.buf[:, self.offsets[i]:self.offsets[i] + self.widths[i]]

    def record(self, i: int, out: torch.Tensor, node) -> None:
        self.written[i] = (out, node)

    def cat(self, xs: List[torch.Tensor]) -> torch.Tensor:
        if self.buf is None or not self.written:
            return torch.cat(xs, dim=1)
        return _CatSinkFn.apply(self, *xs)


class _CatSinkFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, sink: ConcatSink, *xs):
        nodes = []
        for i, x in enumerate(xs):
            hit = sink.written.get(i)
            if hit is not None and hit[0] is x:
                nodes.append(hit[1])
            else:  # a branch no fused kernel stored (STDC's pooled x1): copy it in
                sink.buf[:, sink.offsets[i]:sink.offsets[i] + sink.widths[i]].copy_(x)
                nodes.append(None)
        # the node keeps only the slice geometry and the BN nodes: the buffer (about to carry this
        # node as its grad_fn) and the branch outputs are released from the sink -- no
        # tensor -> grad_fn -> sink -> tensor reference cycle holding GPU memory until a GC pass
        ctx.geom, ctx.nodes = list(zip(sink.offsets, sink.widths)), nodes
        ctx.set_materialize_grads(False)
        out, sink.buf, sink.written = sink.buf, None, {}
        return out

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return (None,) * (1 + len(ctx.nodes))
        cl = g.is_contiguous(memory_format=torch.channels_last) and g.data_ptr() % 16 == 0
        grads = []
        for (off, width), node in zip(ctx.geom, ctx.nodes):
            sl = g[:, off:off + width]
            if cl and node is not None and getattr(node, "dy2_slot", None) is not None:
                node.dy2_slot.append(sl)  # the BN backward reads it in place
                grads.append(None)
            else:
                grads.append(sl)
        return (None, *grads)
