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
        self.pooled: dict = {}  # branch index -> (kernel, stride, padding) of a PooledPart

    def slot(self, i: int, like: torch.Tensor) -> Optional[torch.Tensor]:
        """Channel slice ``i`` of the buffer for a branch output shaped like ``like`` (allocated
        on first use), or None when the fused kernels cannot store there."""
        if like.dim() != 4 or not like.is_cuda:
            return None
        return self._slot(i, tuple(like.shape), like.dtype, like.device)

    def _slot(self, i, shape, dtype, device) -> Optional[torch.Tensor]:
        n, c, h, w = shape
        if c != self.widths[i] or not _ENABLED:
            return None
        if torch.onnx.is_in_onnx_export() or torch.jit.is_tracing():
            return None  # exported graphs keep the plain cat
        vec = 128 // torch.finfo(dtype).bits
        if self.offsets[i] % vec or self.total % vec or self.widths[i] % vec or self.widths[i] // vec > 256:
            return None
        if self.buf is None:
            self.buf = torch.empty((n, self.total, h, w), dtype=dtype, device=device,
                                   memory_format=torch.channels_last)
        elif self.buf.dtype != dtype or self.buf.shape[0] != n or tuple(self.buf.shape[2:]) != (h, w):
            return None
        return self.buf[:, self.offsets[i]:self.offsets[i] + self.widths[i]]

    def max_pool(self, i: int, x: torch.Tensor, kernel_size: int, stride: int, padding: int = 0,
                 dtype: Optional[torch.dtype] = None):
        """Branch ``i`` = ``max_pool2d(x, kernel_size, stride, padding)``, pooled by the cat node
        itself straight into its channel slice (:class:`PooledPart`; the pool kernel indexes its
        output by strides, ``pool2d_fwd_out``) -- or the pooled tensor when that path is off.
        ``dtype``: the concat's dtype (autocast: a bf16 conv branch next to a pooled fp32 image);
        a pool input of another dtype takes the tensor path, cast to it."""
        from .pool import _hip_ok, max_pool2d

        k, s, p = int(kernel_size), int(stride), int(padding)
        if dtype is not None and x.dtype != dtype:
            return max_pool2d(x, k, s, p).to(dtype)
        if x.dim() == 4 and x.is_cuda and _hip_ok(x) and x.dtype != torch.float16:
            n, c, h, w = x.shape
            shape = (n, c, (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1)
            if self._slot(i, shape, x.dtype, x.device) is not None:
                self.pooled[i] = (k, s, p)
                return PooledPart(x, k, s, p)
        return max_pool2d(x, k, s, p)

    def record(self, i: int, out: torch.Tensor, node) -> None:
        self.written[i] = (out, node)

    def cat(self, xs: List[torch.Tensor]) -> torch.Tensor:
        if self.buf is None or not (self.written or self.pooled):
            return torch.cat([x.materialize() if isinstance(x, PooledPart) else x for x in xs], dim=1)
        return _CatSinkFn.apply(self, *[x.x if isinstance(x, PooledPart) else x for x in xs])


class PooledPart:
    """A max-pool concat branch that the cat node computes into its buffer slice (no pooled
    tensor, no cat read of it; backward: the pool backward reads the slice of the cat's gradient
    at its row stride)."""
    __slots__ = ("x", "k", "s", "p")

    def __init__(self, x, k, s, p):
        self.x, self.k, self.s, self.p = x, k, s, p

    def materialize(self) -> torch.Tensor:
        from .pool import max_pool2d

        return max_pool2d(self.x, self.k, self.s, self.p)


class _CatSinkFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, sink: ConcatSink, *xs):
        nodes, pools = [], {}
        for i, x in enumerate(xs):
            hit = sink.written.get(i)
            sl = sink.buf[:, sink.offsets[i]:sink.offsets[i] + sink.widths[i]]
            if i in sink.pooled:  # x is the pool's input: pooled straight into the slice
                k, s, p = sink.pooled[i]
                idx = _ops().pool2d_fwd_out(x, sl, [k, k], [s, s], [p, p], 1, True)
                pools[i] = (idx, x.shape[2], x.shape[3], k, s, p)
                nodes.append(None)
            elif hit is not None and hit[0] is x:
                nodes.append(hit[1])
            else:  # a branch no fused kernel stored (STDC's pooled x1): copy it in
                sl.copy_(x)
                nodes.append(None)
        # the node keeps only the slice geometry and the BN nodes: the buffer (about to carry this
        # node as its grad_fn) and the branch outputs are released from the sink -- no
        # tensor -> grad_fn -> sink -> tensor reference cycle holding GPU memory until a GC pass
        ctx.geom, ctx.nodes, ctx.pools = list(zip(sink.offsets, sink.widths)), nodes, pools
        ctx.set_materialize_grads(False)
        out, sink.buf, sink.written, sink.pooled = sink.buf, None, {}, {}
        return out

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return (None,) * (1 + len(ctx.nodes))
        cl = g.is_contiguous(memory_format=torch.channels_last) and g.data_ptr() % 16 == 0
        grads = []
        for i, ((off, width), node) in enumerate(zip(ctx.geom, ctx.nodes)):
            sl = g[:, off:off + width]
            if i in ctx.pools:  # the max-pool backward reads the slice at its row stride
                idx, h, w, k, s, p = ctx.pools[i]
                grads.append(_ops().pool2d_bwd(sl, idx, h, w, [k, k], [s, s], [p, p], 1, True))
            elif cl and node is not None and getattr(node, "dy2_slot", None) is not None:
                node.dy2_slot.append(sl)  # the BN backward reads it in place
                grads.append(None)
            else:
                grads.append(sl)
        return (None, *grads)


# --------------------------------------------------------------------------- concat -> BN
# ``act(bn(torch.cat(parts, 1)))`` -- CGNet's joint feature (loc || sur, reference
# models/cgnet.py:90-110), EDANet's / ENet-family downsamplers (conv || pool, edanet.py:26-45):
# BatchNorm is per channel, so the concat's statistics are the parts' statistics side by side and
# each part can be normalised straight into its channel slice of the output.  Forward: per-part
# statistics (``bn_stats_sums``), ONE finalize over the joined sums (running stats updated once),
# per-part apply into the output slice (``bn_apply(slice_only=True)``); backward: per-part BN
# backward reading its slice of the output gradient at the row stride (``grad2``).  No concat is
# materialised either way, and the parts' gradients are never slice copies.
from .bn import (ACT_NONE, MASK_FROM_X, MASK_NONE, _aligned_cl, _sync_group, act_code,  # noqa: E402
                 bump_write_generation, eval_coeffs, fused_ok)
from ._ext import ops as _ops, use_hip as _use_hip  # noqa: E402

CAT_BN_CALLS = [0]  # forward passes that took the fused path (tests)


def _cat_bn_ok(parts, bn, code) -> bool:
    if not _ENABLED or len(parts) < 2 or not _use_hip(parts[0], "bn") or code not in (0, 1, 2):
        return False
    if torch.onnx.is_in_onnx_export() or torch.jit.is_tracing():
        return False
    p0 = parts[0]
    if p0.dim() != 4 or p0.dtype not in (torch.bfloat16, torch.float32) or not fused_ok(p0, bn, code):
        return False
    if _sync_group(bn) is not None:
        return False
    vec = 16 // p0.element_size()
    off = 0
    for p in parts:
        if (p.dim() != 4 or p.dtype != p0.dtype or p.device != p0.device or p.shape[0] != p0.shape[0]
                or p.shape[2:] != p0.shape[2:] or p.shape[1] % vec or p.shape[1] // vec > 256):
            return False
        off += p.shape[1]
    return off == bn.num_features and off % vec == 0


class _CatBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, bn, code, weight, bias, *parts):
        parts = tuple(_aligned_cl(p) for p in parts)
        n, h, w = parts[0].shape[0], parts[0].shape[2], parts[0].shape[3]
        widths = [p.shape[1] for p in parts]
        offs = [sum(widths[:i]) for i in range(len(widths))]
        c = sum(widths)
        out = torch.empty((n, c, h, w), dtype=parts[0].dtype, device=parts[0].device,
                          memory_format=torch.channels_last)
        use_batch = bn.training or not bn.track_running_stats or bn.running_mean is None
        if use_batch:
            track = bn.track_running_stats and bn.training and bn.running_mean is not None
            ps = [_ops().bn_stats_sums(p) for p in parts]  # [2Cp + 1]: sum, second moment, count
            sums = torch.cat([s[:cp] for s, cp in zip(ps, widths)] + [s[cp:2 * cp] for s, cp in zip(ps, widths)]
                             + [ps[0][-1:]])
            mi, ss = _ops().bn_finalize(sums, weight, bias, bn.running_mean if track else None,
                                        bn.running_var if track else None,
                                        bn.num_batches_tracked if track else None, float(bn.momentum), float(bn.eps))
            if track:
                bump_write_generation()  # running stats rewritten through raw pointers
        else:
            sums = None
            mi, ss = eval_coeffs(bn)

        def sl(t, o, cp):  # [2C] -> the part's [2Cp] (first half, second half)
            return torch.cat((t[o:o + cp], t[c + o:c + o + cp]))

        for p, o, cp in zip(parts, offs, widths):
            _ops().bn_apply(p, sl(ss, o, cp), None, code, out[:, o:o + cp], True)
        CAT_BN_CALLS[0] += 1
        ctx.widths, ctx.offs, ctx.code, ctx.use_batch, ctx.c = widths, offs, code, use_batch, c
        ctx.has_w = weight is not None
        ctx.save_for_backward(mi, ss, sums, weight, *parts)
        return out

    @staticmethod
    def backward(ctx, g):
        mi, ss, sums, weight, *parts = ctx.saved_tensors
        g = _aligned_cl(g)
        c = ctx.c
        mask = MASK_NONE if ctx.code == ACT_NONE else MASK_FROM_X
        want_dw = ctx.has_w and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        dxs, dws, dbs = [], [], []

        def sl(t, o, cp):
            return torch.cat((t[o:o + cp], t[c + o:c + o + cp]))

        for i, (p, o, cp) in enumerate(zip(parts, ctx.offs, ctx.widths)):
            sums_p = torch.cat((sums[o:o + cp], sums[c + o:c + o + cp], sums[2 * c:])) if sums is not None else None
            w_p = weight[o:o + cp] if weight is not None else None
            dx, _, dw, db = _ops().bn_backward(None, p, None, None, sums_p, sl(mi, o, cp), sl(ss, o, cp), w_p,
                                               ctx.code, mask, False, ctx.use_batch, want_dw, None, g[:, o:o + cp])
            dxs.append(dx if ctx.needs_input_grad[4 + i] else None)
            dws.append(dw)
            dbs.append(db)
        dwt = torch.cat(dws).to(weight.dtype) if want_dw else None
        dbt = torch.cat(dbs).to(weight.dtype) if want_dw else None
        return (None, None, dwt if ctx.needs_input_grad[2] else None, dbt if ctx.needs_input_grad[3] else None,
                *dxs)


def cat_bn_act(parts, bn, act=None, act_module=None):
    """``act(bn(torch.cat(parts, dim=1)))`` without the concat (see above); ``act``: a fused
    activation (code / str / module) -- any other activation module runs on the BN output."""
    code = act if isinstance(act, int) else act_code(act)
    post = None
    if code is None:  # e.g. PReLU: the BN into the concat layout, then the activation module
        code, post = ACT_NONE, (act_module if act_module is not None else act)
    parts = list(parts)
    if parts[0].is_cuda and any(p.dtype != parts[0].dtype for p in parts):
        dt = parts[0].dtype
        for p in parts[1:]:
            dt = torch.promote_types(dt, p.dtype)
        parts = [p.to(dt) for p in parts]
    if _cat_bn_ok(parts, bn, code):
        y = _CatBNFn.apply(bn, code, bn.weight, bn.bias, *parts)
    else:
        from .bn import bn_act

        y = bn_act(torch.cat(parts, dim=1), bn, code)
    return post(y) if post is not None else y
