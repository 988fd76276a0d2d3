"""Fused BatchNorm (+ residual) + activation, with SyncBN over RCCL (HIP ``bn_act.hip``).

``bn_act(x, bn, act, residual)`` computes ``act(BN(x) + residual)`` for a
``nn.BatchNorm2d`` / ``nn.SyncBatchNorm`` module ``bn`` (its running stats and
``num_batches_tracked`` are updated exactly like PyTorch's).  GPU fast path
conditions: channels-last activations, any C whose widest dividing channel
vector (16/8/4 bytes or one element) leaves <= 256 vectors per row,
activation in {none, relu, relu6}, ``momentum`` not None; anything
else runs the stock PyTorch modules.

SyncBN: per-channel (sum, sum of squares, count) are produced in fp64 by one
reduction kernel and summed across ranks with ONE ``all_reduce`` of 2C+1
doubles (backward: one all-reduce of 2C doubles) on the current stream -- the
reference's SyncBatchNorm all-gathers mean/invstd/count instead.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ._ext import bump_write_generation, use_hip, ops, write_generation

ACT_NONE, ACT_RELU, ACT_RELU6 = 0, 1, 2
MASK_NONE, MASK_FROM_Y, MASK_FROM_X, MASK_BITS = 0, 1, 2, 3
# residual + activation: the forward writes a 1-bit-per-element activation-derivative mask
# (MASK_BITS) instead of the backward re-reading the bf16 output y twice (RTSEG_BN_BITS=0: off)
_USE_BITS = os.environ.get("RTSEG_BN_BITS", "1") != "0"
# residual-gradient hand-off to the upstream conv's dgrad (RTSEG_RES_HANDOFF=0: off, for A/B)
_HANDOFF = os.environ.get("RTSEG_RES_HANDOFF", "1") != "0"
# ... as the BN output's gradient + its activation bit mask, applied in the dgrad epilogue, so the
# BN backward never writes the masked residual gradient.  Opt-in (RTSEG_MASKED_HANDOFF=1): on the
# DDRNet-23 b32 step it measured 0.7 % slower than writing the masked gradient out (524.8 / 524.4
# vs 528.5 images/s, profiles/r5_masked) -- the epilogue's per-lane mask-byte loads cost more
# than the saved 2-byte-per-element write
_MASKED_HANDOFF = os.environ.get("RTSEG_MASKED_HANDOFF", "0") == "1"
# the stem BN's forward apply as a recompute of the stem conv (RTSEG_STEM_BN_RECOMPUTE=0: off, A/B)
_STEM_BN_RECOMPUTE = os.environ.get("RTSEG_STEM_BN_RECOMPUTE", "1") != "0"
# single-GPU BN backward started early on a side stream by the consumer conv (bn_bwd_early).
# Opt-in (RTSEG_BN_OVERLAP=1): bitwise equal, but DDRNet-23 b32 measured 573.3 / 575.0 images/s with
# it against 578.6 / 579.5 without on one box (profiles/r6_negative). The memory-bound BN passes slow
# the weight-gradient kernels they share the CUs with more than they hide.
_OVERLAP = os.environ.get("RTSEG_BN_OVERLAP", "0") == "1"


def act_code(act) -> Optional[int]:
    """Activation module/str -> fused code, or None when it cannot be fused."""
    if act is None:
        return ACT_NONE
    if isinstance(act, str):
        return {"none": ACT_NONE, "relu": ACT_RELU, "relu6": ACT_RELU6}.get(act.lower())
    inner = getattr(act, "activation", act)  # models.modules.Activation wrapper
    if isinstance(inner, nn.Identity):
        return ACT_NONE
    if isinstance(inner, nn.ReLU6):
        return ACT_RELU6
    if isinstance(inner, nn.ReLU):
        return ACT_RELU
    if isinstance(inner, nn.Hardtanh) and inner.min_val == 0.0 and inner.max_val == 6.0:
        return ACT_RELU6
    return None


def _sync_group(bn):
    if not isinstance(bn, nn.SyncBatchNorm):
        return None
    if not (dist.is_available() and dist.is_initialized()):
        return None
    pg = bn.process_group or dist.group.WORLD
    return pg if dist.get_world_size(pg) > 1 else None


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, bn, act, use_batch_stats, pg, part=None, out2=None, pending=None):
        if use_batch_stats:
            track = bn.track_running_stats and bn.training and bn.running_mean is not None
            rm = bn.running_mean if track else None
            rv = bn.running_var if track else None
            nb = bn.num_batches_tracked if track else None
            count = float(x.numel() // x.shape[1])
            if pg is None:
                if part is not None:  # statistics already produced by the conv epilogue
                    mi, ss, sums = ops().bn_finalize_slab(part, weight, bias, rm, rv, nb, float(bn.momentum),
                                                          float(bn.eps), count)
                else:
                    mi, ss, sums = ops().bn_stats_finalize(x, weight, bias, rm, rv, nb,
                                                           float(bn.momentum), float(bn.eps))
            else:  # SyncBN: one all-reduce of (sum, sumsq, count) in fp64 over RCCL
                if pending is not None:  # issued by bn_stats_begin (async): wait for it here
                    sums, work = pending
                else:  # issued here, asynchronously as everywhere: the wait is the finalize's dependency
                    sums = ops().bn_slab_sums(part, count) if part is not None else ops().bn_stats_sums(x)
                    work = dist.all_reduce(sums, group=pg, async_op=True)
                work.wait()
                mi, ss = ops().bn_finalize(sums, weight, bias, rm, rv, nb, float(bn.momentum),
                                           float(bn.eps))
            if rm is not None:
                # the finalize kernels rewrite running_mean / running_var through raw pointers
                # (no _version bump): invalidate the eval-coefficient caches keyed on them
                bump_write_generation()
        else:
            sums = None
            mi, ss = eval_coeffs(bn)
        if act == ACT_NONE:
            mask = MASK_NONE
        elif residual is None:
            mask = MASK_FROM_X
        else:
            mask = MASK_BITS if _USE_BITS else MASK_FROM_Y
        # a stem conv produced x (batch statistics, no residual / concat slice): the apply is a
        # recompute of that K = 27 conv from the 0.4 GB image with the BN + act epilogue on its
        # fp32 accumulators (conv_stem_bn_act) -- no pass over the 2.1 GB x
        sprod = x.grad_fn if (use_batch_stats and residual is None and out2 is None and _STEM_BN_RECOMPUTE
                              and mask in (MASK_NONE, MASK_FROM_X) and x.dtype == torch.bfloat16) else None
        stem_io = getattr(sprod, "stem_io", None)
        # out2: this output's channel slice of a concat buffer (ops/concat.py), stored too
        if stem_io is not None:
            xi, wk, st, pd, dl = stem_io
            y, bits = ops().conv_stem_bn_act(xi, wk, st, pd, dl, ss, act), None
            STEM_RECOMPUTES[0] += 1
        elif not getattr(x.grad_fn, "y_stored", True):  # (never expected) give x its values first
            _stem_materialize(x.grad_fn, x)
            y, bits = ops().bn_apply(x, ss, residual, act, out2), None
        elif mask == MASK_BITS:
            y, bits = ops().bn_apply_bits(x, ss, residual, act, out2)
        else:
            y, bits = ops().bn_apply(x, ss, residual, act, out2), None
        # the concat node hands its gradient slice over here (read in place by the kernels)
        ctx.dy2_slot = [] if out2 is not None else None
        ctx.set_materialize_grads(False)
        ctx.act, ctx.mask, ctx.pg = act, mask, pg
        # SyncBN: the consumer conv's backward may issue this node's gradient all-reduce early,
        # between its data and weight gradients (syncbn_bwd_early), and park it here
        # Single GPU: the consumer conv may run this node's whole backward early, on a side stream
        # under its weight gradient (bn_bwd_early). This covers BNs without a residual, concat slice
        # or stem hand-off, i.e. an RB's conv1 -> BN -> ReLU -> conv2.
        overlap = (_OVERLAP and pg is None and residual is None and out2 is None and x.is_cuda
                   and use_batch_stats and x.dtype == torch.bfloat16)
        ctx.early = ([] if (pg is not None or overlap) and not getattr(bn, "_rtseg_no_early", False)
                     else None)
        ctx.bn_module = bn if (pg is not None or overlap) else None
        # a stem conv produced x (ops/conv.py bn_fuse_slot): this node's dx pass moves into that
        # conv's weight gradient (conv_stem_wgrad_bn)
        prod = x.grad_fn if use_batch_stats and residual is None and out2 is None else None
        ctx.stem_node = (prod if getattr(prod, "bn_fuse_slot", None) is not None
                         and mask in (MASK_NONE, MASK_FROM_X) and act in (ACT_NONE, ACT_RELU, ACT_RELU6)
                         else None)
        ctx.batch_stats = use_batch_stats
        ctx.has_res = residual is not None
        # residual add whose residual is the input of an upstream routed conv (DDRNet's RB, ResNet
        # BasicBlock): hand the residual gradient to that conv, whose dgrad epilogue adds it --
        # autograd's separate gradient-accumulation add over the whole tensor disappears
        ctx.handoff = None
        if residual is not None and residual.requires_grad and _HANDOFF:
            from .conv import find_conv_consumer

            node = find_conv_consumer(x, residual)
            if node is not None and node.addend_slot is None:
                node.addend_slot = ctx.handoff = []
        ctx.has_w = weight is not None
        ctx.save_for_backward(x, y if mask == MASK_FROM_Y else bits, mi, ss, sums, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mi, ss, sums, weight = ctx.saved_tensors
        mask = ctx.mask
        dy2 = ctx.dy2_slot.pop() if ctx.dy2_slot else None
        if dy is None and dy2 is None:
            return (None,) * 11
        dy_in = dy  # (as autograd passed it: the early SyncBN reduction is matched on it)
        if dy is not None:
            dy = _aligned_cl(dy)
        bsums = local = None
        want_dres = ctx.has_res and ctx.needs_input_grad[3]
        want_dw = ctx.has_w and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        stem, ctx.stem_node = ctx.stem_node, None
        if stem is not None and dy is not None and dy2 is None and ctx.needs_input_grad[0]:
            return _stem_handoff(ctx, stem, dy, x, y, mi, ss, sums, weight, want_dw)
        if not getattr(x.grad_fn, "y_stored", True):
            # a stats-only stem launch (RTSEG_STEM_NO_STORE=1) never wrote x, and this backward
            # reads it (the hand-off above was not taken: a second backward, another consumer)
            _stem_materialize(x.grad_fn, x)
        if ctx.pg is None and ctx.early:  # the whole backward ran early on the side stream
            key, res, ev = ctx.early.pop()
            torch.cuda.current_stream(dy_in.device if dy_in is not None else None).wait_event(ev)
            if dy2 is None and _same_grad(dy_in, key):
                e_dx, e_dw, e_db = res
                EARLY_USED[0] += 1
                return (e_dx, e_dw, e_db, None, None, None, None, None, None, None, None)
            ctx.bn_module._rtseg_no_early = True  # another consumer's gradient was added: not again
        if ctx.pg is not None:
            early = ctx.early.pop() if ctx.early else None
            if early is not None:
                key, e_sums, e_local, work = early
                work.wait()
                if dy2 is None and _same_grad(dy_in, key):
                    bsums, local = e_sums, e_local  # reduced while the consumer's wgrad ran
                else:
                    # the output had another consumer (its gradient is a sum): this site never
                    # issues early again -- every rank sees the same graph, so decides the same
                    ctx.bn_module._rtseg_no_early = True
            if bsums is None:
                bsums = ops().bn_bwd_sums(dy, x, y, mi, ss, ctx.act, mask, dy2)
                if want_dw:
                    local = bsums.clone()
                dist.all_reduce(bsums, group=ctx.pg)
        # the residual gradient dy * act'(z) handed over unmaterialised: the conv's dgrad epilogue
        # applies the bit mask to dy itself (ops/conv.py MaskedAddend) -- no dres write here
        masked = (want_dres and ctx.handoff is not None and mask == MASK_BITS and dy is not None
                  and dy2 is None and _MASKED_HANDOFF and x.dtype == torch.bfloat16
                  and x.shape[1] % 8 == 0 and x.shape[1] <= 2048)  # one mask byte per 8 channels
        dx, dres, dw, db = ops().bn_backward(dy, x, y, bsums, sums, mi, ss, weight, ctx.act,
                                             mask, want_dres and not masked, ctx.batch_stats, want_dw, None, dy2)
        if masked:
            from .conv import MaskedAddend

            dres = MaskedAddend(dy, y)  # y holds the activation bits (MASK_BITS)
            MASKED_HANDOFFS[0] += 1
        if local is not None:
            # parameter gradients are this rank's contribution (DDP averages them), as in torch's
            # SyncBatchNorm; only the input-gradient coefficients use the all-reduced sums
            c = local.numel() // 2
            dw = (local[c:] * mi[c:].double()).float()
            db = local[:c].float()
        if want_dres and ctx.handoff is not None:
            ctx.handoff.append(dres)  # the conv node adds it in its dgrad epilogue
            dres = None
        return (dx, dw if want_dw else None, db if want_dw else None,
                dres if want_dres else None, None, None, None, None, None, None, None)


MASKED_HANDOFFS = [0]  # residual gradients handed over as (gradient, bit mask) (tests)
STEM_RECOMPUTES = [0]  # stem BN forward applies run as conv_stem_bn_act (tests)
STEM_HANDOFFS = [0]  # BN backward dx passes handed to a stem conv's weight gradient (tests)


def _stem_materialize(node, x: torch.Tensor) -> None:
    """Write a stats-only stem launch's conv output into its (allocated, unwritten) tensor ``x``:
    the fallback for a consumer that needs the stored values after all."""
    xi, wk, st, pd, dl = node.stem_io
    with torch.no_grad():
        x.copy_(ops().conv_stem(xi, wk, st, pd, dl, False)[0])
    node.y_stored = True


def _stem_handoff(ctx, stem, dy, x, y, mi, ss, sums, weight, want_dw):
    """BN backward whose dx pass runs in the producing stem conv's weight gradient: only the
    reduction + finalize here (``bn_bwd_coeffs``), the coefficients handed to the conv node, and a
    zero-stride placeholder returned as dx (no HBM traffic).  On the flagship this is DDRNet-23's
    first BN, at half resolution: the largest tensor of the step (2.1 GB at batch 32)."""
    bsums = local = None
    stem_io = getattr(stem, "stem_io", None)
    recompute = stem_io is not None and _STEM_BN_RECOMPUTE and x.dtype == torch.bfloat16

    def reduce_sums():  # [2C] fp64 (sum g', sum g' (x - mean)) of this rank
        if recompute:  # the conv output recomputed from the image, not read back (conv_stem.hip)
            xi, wk, st, pd, dl = stem_io
            slab = ops().conv_stem_bn_sums(xi, wk, st, pd, dl, dy, mi, ss, ctx.act)
            STEM_RECOMPUTES[0] += 1
            return ops().bn_slab_sums(slab, -1.0)[: 2 * x.shape[1]]
        return ops().bn_bwd_sums(dy, x, y, mi, ss, ctx.act, ctx.mask, None)

    if ctx.pg is not None:  # SyncBN: the reduction is all-reduced as usual (early if issued)
        early = ctx.early.pop() if ctx.early else None
        if early is not None:
            key, e_sums, e_local, work = early
            work.wait()
            if _same_grad(dy, key):
                bsums, local = e_sums, e_local
            else:
                ctx.bn_module._rtseg_no_early = True
        if bsums is None:
            bsums = reduce_sums()
            if want_dw:
                local = bsums.clone()
            dist.all_reduce(bsums, group=ctx.pg)
    elif recompute:
        bsums = reduce_sums()
    k, dw, db = ops().bn_bwd_coeffs(dy, x, y, bsums, sums, mi, ss, weight, ctx.act, ctx.mask,
                                    ctx.batch_stats, want_dw)
    if local is not None:
        c = local.numel() // 2
        dw = (local[c:] * mi[c:].double()).float()
        db = local[:c].float()
    dummy = x.new_zeros(()).expand(x.shape)
    act, mask, batch = ctx.act, ctx.mask, ctx.batch_stats  # (act codes 0 / 1 / 2 = the kernel's)

    def full():  # the plain dx (the conv output had another consumer)
        if not getattr(stem, "y_stored", True):
            _stem_materialize(stem, x)
        return ops().bn_backward(dy, x, y, bsums, sums, mi, ss, weight, act, mask, False, batch, False,
                                 None, None)[0]

    stem.bn_fuse_slot.append((dy, x, k, mi, ss, act, dummy, full))
    STEM_HANDOFFS[0] += 1
    return (dummy, dw if want_dw else None, db if want_dw else None, None, None, None, None, None, None,
            None, None)


EARLY_ISSUED = [0]  # SyncBN backward all-reduces issued early by a consumer conv (tests)
EARLY_OVERLAPPED = [0]  # single-GPU BN backwards started on the side stream (tests)
EARLY_USED = [0]  # ... whose results the BN node returned (tests)
_SIDE = {}


def _side_stream(device) -> torch.cuda.Stream:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _SIDE.get(idx)
    if s is None:
        s = _SIDE[idx] = torch.cuda.Stream(device=idx)
    return s


def bn_bwd_early(node, dy: torch.Tensor) -> bool:
    """Called by the consumer conv's backward right after its data gradient ``dy`` (ops/conv.py):
    multi-rank SyncBN -> :func:`syncbn_bwd_early`; single GPU -> this BN node's whole backward
    (reduction, finalize, dx / dw / db) is launched now on a side stream, so its memory-bound passes
    run beside the conv's compute-bound weight gradient on the main stream. The node's backward
    waits on the event, and it uses the results only if the gradient it receives is exactly ``dy``
    (``_same_grad``: the conv was the output's only consumer)."""
    if getattr(node, "pg", None) is not None:
        return syncbn_bwd_early(node, dy)
    early = getattr(node, "early", None)
    if early is None or early or getattr(node, "dy2_slot", None) is not None or node.has_res:
        return False
    if node.stem_node is not None:
        return False
    x, y, mi, ss, sums, weight = node.saved_tensors
    if (dy.dtype != x.dtype or dy.shape != x.shape or dy.data_ptr() % 16
            or not dy.is_contiguous(memory_format=torch.channels_last)):
        return False
    if not getattr(x.grad_fn, "y_stored", True):
        return False
    want_dw = node.has_w and (node.needs_input_grad[1] or node.needs_input_grad[2])
    main = torch.cuda.current_stream(dy.device)
    side = _side_stream(dy.device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        bsums = ops().bn_bwd_sums(dy, x, y, mi, ss, node.act, node.mask, None)
        dx, _, dw, db = ops().bn_backward(dy, x, y, bsums, sums, mi, ss, weight, node.act, node.mask, False,
                                          node.batch_stats, want_dw, None, None)
        ev = torch.cuda.Event()
        ev.record(side)
    # cross-stream lifetimes: dy / x / y were made on the main stream and are read on the side one;
    # the results are made on the side stream and used on the main one after the event
    for t in (dy, x, y, mi, ss, bsums) + ((sums,) if sums is not None else ()) + ((weight,) if weight is not None else ()):
        if t is not None and t.is_cuda:
            t.record_stream(side)
    for t in (dx, dw, db):
        if t is not None:
            t.record_stream(main)
    early.append(((dy, dy._version), (dx, dw if want_dw else None, db if want_dw else None), ev))
    EARLY_OVERLAPPED[0] += 1
    return True


def syncbn_bwd_early(node, dy: torch.Tensor) -> bool:
    """Issue SyncBN node ``node``'s backward all-reduce now, asynchronously, from the backward
    of the conv that consumes the BN output (ops/conv.py, right after its data gradient ``dy``
    is computed and before its weight gradient): the RCCL round trip then runs under that wgrad
    instead of stalling the stream between ``bn_bwd_sums`` and the dx kernel of every SyncBN layer
    (reference utils/parallel.py:34-43 runs torch's SyncBatchNorm, whose backward all-reduce is
    synchronous).  ``_BNActFn.backward`` waits on it and uses it only if the gradient it receives
    is exactly ``dy`` (the conv was the output's only consumer); otherwise it recomputes.  Every
    rank takes the same decisions (same graph), so the collectives stay matched."""
    early = getattr(node, "early", None)
    if early is None or early or getattr(node, "dy2_slot", None) is not None or node.pg is None:
        return False
    x, y, mi, ss, _, _ = node.saved_tensors
    if (dy.dtype != x.dtype or dy.shape != x.shape or dy.data_ptr() % 16
            or not dy.is_contiguous(memory_format=torch.channels_last)):
        return False
    if not getattr(x.grad_fn, "y_stored", True):
        _stem_materialize(x.grad_fn, x)
    bsums = ops().bn_bwd_sums(dy, x, y, mi, ss, node.act, node.mask, None)
    want_dw = node.has_w and (node.needs_input_grad[1] or node.needs_input_grad[2])
    local = bsums.clone() if want_dw else None
    work = dist.all_reduce(bsums, group=node.pg, async_op=True)
    # the key holds a reference to dy itself: autograd then cannot accumulate another consumer's
    # gradient into dy in place (its input buffer adds in place only into a tensor nobody else
    # holds) -- a sum arrives as a new tensor -- and the version counter catches any other
    # in-place write (_same_grad)
    early.append(((dy, dy._version), bsums, local, work))
    EARLY_ISSUED[0] += 1
    return True


def _same_grad(dy, key) -> bool:
    """Whether the gradient a SyncBN node received is exactly the tensor its consumer conv
    reduced early (``syncbn_bwd_early``), unmodified: same tensor (or storage, shape and strides)
    and same version.  Anything else -- a second consumer's gradient added, in place or not --
    means the early sums are of a partial gradient and must not be used."""
    ref, ver = key
    if dy is None:
        return False
    same = dy is ref or (dy.data_ptr() == ref.data_ptr() and dy.shape == ref.shape
                         and dy.stride() == ref.stride() and dy.dtype == ref.dtype)
    return same and dy._version == ver


def eval_coeffs(bn):
    """(mean_invstd, scale_shift) of an eval-mode BN from its running statistics, cached on
    the module until any of weight / bias / running stats changes (an inference forward --
    and its HIP graph -- then has no per-layer coefficient kernel)."""
    ts = (bn.weight, bn.bias, bn.running_mean, bn.running_var)
    key = tuple((t.data_ptr(), t._version) if t is not None else None for t in ts) + (float(bn.eps),
                                                                                     write_generation())
    hit = getattr(bn, "_rtseg_eval_coeffs", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    out = ops().bn_eval_coeffs(bn.weight, bn.bias, bn.running_mean, bn.running_var, float(bn.eps))
    if not torch.is_grad_enabled():
        bn._rtseg_eval_coeffs = (key, out)
    return out


def vec_width(dtype: torch.dtype, c: int) -> int:
    """Channel-vector width the HIP kernels use (mirror of ``bn_vec_width``); 0 = unsupported."""
    if dtype == torch.float16:
        return 8 if c % 8 == 0 and c // 8 <= 256 else 0
    v = 4 if dtype == torch.float32 else 8
    while v >= 1:
        if c % v == 0 and c // v <= 256:
            return v
        v //= 2
    return 0


def _aligned_cl(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous(memory_format=torch.channels_last) if t.dim() == 4 else t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone(memory_format=torch.channels_last if t.dim() == 4
                                                      else torch.contiguous_format)


def fused_ok(x: torch.Tensor, bn, act) -> bool:
    if not isinstance(bn, (nn.BatchNorm2d, nn.SyncBatchNorm)) or x.dim() != 4:
        return False
    if act is None or bn.momentum is None:
        return False
    if x.dtype not in (torch.float32, torch.bfloat16, torch.float16):
        return False
    if vec_width(x.dtype, x.shape[1]) == 0 or x.numel() == 0:
        return False
    if not x.is_contiguous(memory_format=torch.channels_last) or x.data_ptr() % 16:
        return False
    use_batch = bn.training or not bn.track_running_stats or bn.running_mean is None
    if not use_batch and bn.running_var is None:
        return False
    return bn.affine or bn.weight is None


def bn_stats_begin(x: torch.Tensor, bn, part: Optional[torch.Tensor] = None):
    """Start the SyncBN batch statistics of ``x`` (the BN input) ahead of ``bn_act``: the local fp64
    sums and their all-reduce with ``async_op=True`` -- RCCL runs it on its own stream while the
    caller queues independent work (DDRNet's bilateral fusion: the other branch's conv) -- and
    ``bn_act(..., pending=...)`` waits right before its finalize kernel.  None when ``bn`` is not
    a multi-rank SyncBN on the fused path (``bn_act`` then runs as usual)."""
    if not (use_hip(x, "bn") and fused_ok(x, bn, ACT_NONE)):
        return None
    if not (bn.training or not bn.track_running_stats or bn.running_mean is None):
        return None
    pg = _sync_group(bn)
    if pg is None:
        return None
    count = float(x.numel() // x.shape[1])
    sums = ops().bn_slab_sums(part, count) if part is not None else ops().bn_stats_sums(x)
    return sums, dist.all_reduce(sums, group=pg, async_op=True)


BN_PRELU_FUSED = [0]  # inference BN + PReLU passes run as one kernel (tests)


def _bn_prelu_eval(x: torch.Tensor, bn, act_module) -> Optional[torch.Tensor]:
    """Inference ``prelu(bn_running(x))`` in one pass (act.hip with the BN scale / shift applied
    first), for a per-channel PReLU -- ESPNet-style models run BN then PReLU after every conv, two
    full passes and two launches each at batch 1 (profiles/r6_zoo_latency).  None -> stock path."""
    m = getattr(act_module, "activation", act_module)  # models.modules.Activation wraps it
    if not isinstance(m, nn.PReLU) or torch.is_grad_enabled() or not x.is_cuda or x.dim() != 4:
        return None
    if bn.training or not bn.track_running_stats or bn.running_mean is None or not isinstance(
            bn, (nn.BatchNorm2d, nn.SyncBatchNorm)):
        return None
    w = m.weight
    c = x.shape[1]
    if w.numel() not in (1, c) or w.dtype != torch.float32 or x.dtype not in (torch.float32, torch.bfloat16,
                                                                                 torch.float16):
        return None
    if w.numel() != c:  # a scalar PReLU (the ConvBNAct default): its slope per channel, cached
        key = (w.data_ptr(), w._version, c, write_generation())
        hit = getattr(m, "_rtseg_wc", None)
        if hit is None or hit[0] != key:
            hit = (key, w.detach().reshape(1).expand(c).contiguous())
            m._rtseg_wc = hit
        w = hit[1]
    if not (x.is_contiguous() or x.is_contiguous(memory_format=torch.channels_last)) or x.numel() >= 2 ** 32:
        return None
    if not use_hip(x, "act"):
        return None
    BN_PRELU_FUSED[0] += 1
    return ops().bn_prelu_fwd(x, w.contiguous(), eval_coeffs(bn)[1])


def bn_act(x: torch.Tensor, bn, act=None, residual: Optional[torch.Tensor] = None,
           act_module: Optional[nn.Module] = None, part: Optional[torch.Tensor] = None,
           sink=None, pending=None) -> torch.Tensor:
    """``act(bn(x) + residual)``; ``act`` is a fused-activation code or module/str.

    ``part``: BN statistics slab of ``x`` already computed by its producer (the MFMA conv
    epilogue, ``ops.conv``); used only on the fused batch-statistics path.
    ``sink``: ``(ConcatSink, branch index)`` -- the output is a branch of a channel concat
    (ops/concat.py); the fused kernel also stores it into the concat buffer.
    ``pending``: :func:`bn_stats_begin`'s in-flight SyncBN statistics of ``x``."""
    code = act if isinstance(act, int) else act_code(act)
    if use_hip(x, "bn") and code is not None and fused_ok(x, bn, code) and (
            residual is None or (residual.shape == x.shape
                                 and residual.is_contiguous(memory_format=torch.channels_last)
                                 and residual.data_ptr() % 16 == 0)):
        if residual is not None and residual.dtype != x.dtype:
            residual = residual.to(x.dtype)
        use_batch = bn.training or not bn.track_running_stats or bn.running_mean is None
        pg = _sync_group(bn) if use_batch else None
        out2 = sink[0].slot(sink[1], x) if sink is not None and sink[0] is not None else None
        y = _BNActFn.apply(x, bn.weight, bn.bias, residual, bn, code, use_batch, pg,
                           part if use_batch else None, out2, pending if pg is not None else None)
        if out2 is not None:
            sink[0].record(sink[1], y, y.grad_fn)
        return y
    if pending is not None:
        pending[1].wait()  # (stock path: the statistics are recomputed by the module)
    if act_module is not None and residual is None and sink is None:
        y = _bn_prelu_eval(x, bn, act_module)
        if y is not None:
            return y
    y = bn(x)
    if residual is not None:
        y = y + residual
    if act_module is not None:
        return act_module(y)
    if code == ACT_RELU:
        return torch.relu(y)
    if code == ACT_RELU6:
        return torch.nn.functional.relu6(y)
    if code == ACT_NONE:
        return y
    if callable(act):
        return act(y)
    raise ValueError(f"unsupported activation {act!r}")


def channel_sum(t: torch.Tensor) -> torch.Tensor:
    """fp32 per-channel sum over (N, H, W) -- a bias gradient.  On channels-last GPU tensors it is
    the BN statistics pass (one read, 16-byte chunks, fp64 totals): PyTorch's own reduction over
    the outer dims of a channels-last [N, 19, 1024, 2048] tensor took 63 ms per call on MI355X
    (the x8 transposed-conv heads of CANet / ADSCNet, profiles/r3_models)."""
    if (use_hip(t, "bn") and t.dim() == 4 and t.dtype in (torch.float32, torch.bfloat16) and t.numel() > 0
            and vec_width(t.dtype, t.shape[1]) and t.is_contiguous(memory_format=torch.channels_last)
            and t.data_ptr() % 16 == 0):
        return ops().bn_stats_sums(t)[: t.shape[1]].float()  # shifted, compensated sums (bn_act.hip)
    return t.float().sum((0, 2, 3))


class _BiasAddFn(torch.autograd.Function):
    """y + bias (per channel); the bias gradient is :func:`channel_sum` of dy."""

    @staticmethod
    def forward(ctx, y, bias):
        ctx.bdtype = bias.dtype
        return y + bias.to(y.dtype).view(1, -1, 1, 1)

    @staticmethod
    def backward(ctx, dy):
        return dy, channel_sum(dy).to(ctx.bdtype)


def bias_add(y: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """A conv's bias, added after the bias-free conv: PyTorch's own bias-gradient reduction over a
    channels-last activation ran as a slow non-vectorised reduce (2.3-2.4 ms per LEDNet / ContextNet
    training step at batch 8, profiles/r4_zoo_models); here it is the BN statistics pass."""
    if use_hip(y, "bn") and y.dim() == 4 and bias.dim() == 1 and bias.numel() == y.shape[1]:
        return _BiasAddFn.apply(y, bias)
    return y + bias.view(1, -1, 1, 1)


# --------------------------------------------------------------------------
# Module-level routing: every BatchNorm2d of a model through the fused kernels.
# --------------------------------------------------------------------------
class FusedBatchNorm2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` whose forward runs the HIP kernels when possible.

    Models call ``ops.bn_act`` at their conv-BN-act tails; BatchNorms that are
    used as plain modules (``nn.Sequential(conv, BN, act)`` executed as a
    Sequential, SMP-style blocks, attention branches on pooled maps) are routed
    here by :func:`convert_batchnorm`.  Same parameters / buffers / state_dict.
    """

    def forward(self, x):
        if use_hip(x, "bn") and fused_ok(x, self, ACT_NONE):
            use_batch = self.training or not self.track_running_stats or self.running_mean is None
            pg = _sync_group(self) if use_batch else None
            return _BNActFn.apply(x, self.weight, self.bias, None, self, ACT_NONE, use_batch, pg, None, None, None)
        return nn.BatchNorm2d.forward(self, x)


class FusedSyncBatchNorm(nn.SyncBatchNorm):
    def forward(self, x):
        if use_hip(x, "bn") and fused_ok(x, self, ACT_NONE):
            use_batch = self.training or not self.track_running_stats or self.running_mean is None
            pg = _sync_group(self) if use_batch else None
            return _BNActFn.apply(x, self.weight, self.bias, None, self, ACT_NONE, use_batch, pg, None, None, None)
        return nn.SyncBatchNorm.forward(self, x)


def convert_batchnorm(model: nn.Module) -> nn.Module:
    """Swap the class of every BatchNorm2d / SyncBatchNorm in ``model`` to the fused
    variant (in place; parameters, buffers and checkpoint keys are unchanged)."""
    for m in model.modules():
        if type(m) is nn.BatchNorm2d:
            m.__class__ = FusedBatchNorm2d
        elif type(m) is nn.SyncBatchNorm:
            m.__class__ = FusedSyncBatchNorm
    return model
