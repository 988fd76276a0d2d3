"""Fused optimizer step + model-EMA update (HIP kernel ``csrc/kernels/optim.hip``).

Parity: reference utils/optimizer.py:4-20 (torch SGD / Adam / AdamW) and
utils/model_ema.py:28-40 (EMA lerp with decay ``itrs / total_itrs`` after every
optimizer step).  ``FusedSGD`` / ``FusedAdam`` / ``FusedAdamW`` subclass the
torch optimizers, keep their ``param_groups`` and ``state`` layout (so
checkpoints, ``OneCycleLR`` momentum/beta cycling and ``GradScaler`` work
unchanged) and replace ``step()`` on GPU with ONE multi-tensor launch that also
writes the EMA copy of every parameter when an EMA is attached
(``attach_ema``).  CPU tensors, sparse/complex grads or ``maximize`` /
``amsgrad`` configurations fall back to the stock torch step (then the EMA is
updated separately by ``ModelEmaV2``).
"""
from __future__ import annotations

import math
import os

import torch
from torch.optim import SGD, Adam, AdamW

from ._ext import bump_write_generation, ops, use_hip
from .conv import shadows_written, weight_shadows

MODE_SGD, MODE_ADAM, MODE_ADAMW = 0, 1, 2
META_FIELDS = 14
CHUNK = 16384


def _shadow_fields(p, sh):
    """Meta fields of a conv weight's bf16 shadows (ops/conv.py weight_shadow) or zeros."""
    if sh is None:
        return [0, 0, 0, 0, 0, 0]
    krsc, crsk = sh
    cout, cin, kh, kw = p.shape
    cl = p.dim() == 4 and not p.is_contiguous() and p.is_contiguous(memory_format=torch.channels_last)
    # the data-gradient layout is written after the step by shadow_crsk_tiles' transpose kernel
    crsk_ptr = crsk.data_ptr() if crsk is not None and not _CRSK_TILED else 0
    return [krsc.data_ptr(), crsk_ptr, cout, cin, kh * 256 + kw, 1 if cl else 0]


# RTSEG_CRSK_TILED=0: the fused step writes the CRSK shadow itself (2-byte stores cout apart; A/B)
_CRSK_TILED = os.environ.get("RTSEG_CRSK_TILED", "1") != "0"


def shadow_crsk_tiles(shadows, device):
    """Tile table of ``rtseg.shadow_crsk``: one row per (tap, 64 output x 64 input channels) tile
    of every shadow pair's CRSK layout -> (table, ntiles)."""
    rows = []
    for p, sh in shadows.items():
        if sh is None or sh[1] is None:
            continue
        krsc, crsk = sh
        cout, cin, kh, kw = p.shape
        for rq in range(kh * kw):
            for co0 in range(0, cout, 64):
                for ci0 in range(0, cin, 64):
                    rows += [krsc.data_ptr(), crsk.data_ptr(), cout | (cin << 32), (kh * kw) | (rq << 32),
                             co0 | (ci0 << 32), 0]
    t = torch.tensor(rows, dtype=torch.int64)
    if device.type == "cuda":
        t = t.pin_memory().to(device, non_blocking=True)
    return t, len(rows) // 6


def build_table(rows, device):
    """rows: [(param, grad, state1|None, state2|None, ema|None, first_step[, (krsc, crsk)|None])]
    -> (meta, ntensor, nblocks)."""
    meta, bmap = [], []
    for ti, row in enumerate(rows):
        p, g, s1, s2, e, first = row[:6]
        n = p.numel()
        meta += [p.data_ptr(), g.data_ptr(), s1.data_ptr() if s1 is not None else 0,
                 s2.data_ptr() if s2 is not None else 0, e.data_ptr() if e is not None else 0, n,
                 1 if g.dtype == torch.bfloat16 else 0, 1 if first else 0]
        meta += _shadow_fields(p, row[6] if len(row) > 6 else None)
        for start in range(0, n, CHUNK):
            bmap += [ti, start]
    t = torch.tensor(meta + bmap, dtype=torch.int64)
    if device.type == "cuda":
        # pinned staging + async copy: rebuilding the table never blocks the host on the GPU queue
        t = t.pin_memory().to(device, non_blocking=True)
    return t, len(rows), len(bmap) // 2


def _dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense (some permutation of a contiguous layout)."""
    if t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)):
        return True
    expected = 1
    for st, sz in sorted((st, sz) for sz, st in zip(t.shape, t.stride()) if sz != 1):
        if st != expected:
            return False
        expected *= sz
    return True


def same_layout(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Same shape, both dense, and the same MEMORY order of their size>1 dims -- i.e. walking both
    linearly visits the same elements.  Strides of size-1 dims are irrelevant: a 1x1 conv weight
    is (C,1,C,C) after ``.to(channels_last)`` but (C,1,1,1) when freshly allocated."""
    if a.shape != b.shape:
        return False
    if a.stride() == b.stride():
        return _dense(a)
    if not (_dense(a) and _dense(b)):
        return False
    big = [i for i in range(a.dim()) if a.shape[i] > 1]
    return sorted(big, key=lambda i: -a.stride(i)) == sorted(big, key=lambda i: -b.stride(i))


def _dense_ok(p) -> bool:
    """The kernel walks every tensor of a row linearly in MEMORY order, so param, grad, state
    and EMA only need to be dense in the same memory order (channels-last conv weights are fine)."""
    g = p.grad
    return (p.is_cuda and p.dtype == torch.float32 and g is not None and not g.is_sparse
            and g.dtype in (torch.float32, torch.bfloat16) and same_layout(g, p))


class _FusedMixin:
    """Shared machinery: tensor-table cache, EMA attachment, fallback policy."""

    _mode = MODE_SGD

    def _fused_init(self):
        self._ema_of = {}          # param -> EMA tensor
        self.ema_weight = None     # 1 - decay for the NEXT step (set by the trainer); None => no fused EMA
        self._tables = {}
        self.last_step_fused = False  # parameter EMAs written by this step's launch
        self.fused_steps = 0          # steps that ran the fused kernel (vs the stock torch step)

    def attach_ema(self, pairs):
        """pairs: iterable of (model_param, ema_tensor) of identical shape/dtype/strides."""
        self._ema_of = {p: e for p, e in pairs if same_layout(e, p) and e.dtype == p.dtype}
        self._tables = {}

    def _can_fuse(self, group) -> bool:
        if group.get("maximize", False) or group.get("differentiable", False):
            return False
        if group.get("amsgrad", False) or group.get("capturable", False):
            return False
        ps = [p for p in group["params"] if p.grad is not None]
        return bool(ps) and all(_dense_ok(p) for p in ps) and use_hip(ps[0])

    def _crsk(self, shadows):
        """CRSK shadows of this step's weights (after the step wrote their KRSC shadows)."""
        if not _CRSK_TILED or not shadows:
            return
        key = tuple((sh[0].data_ptr(), sh[1].data_ptr()) for sh in shadows.values() if sh is not None and sh[1] is not None)
        if not key:
            return
        if self._tables.get("crsk", (None,))[0] != key:
            dev = next(iter(shadows.values()))[0].device
            self._tables["crsk"] = (key, shadow_crsk_tiles(shadows, dev))
        table, n = self._tables["crsk"][1]
        ops().shadow_crsk(table, n)

    def _launch(self, slot, rows, hp):
        """One fused launch over ``rows``.  The device pointer table is cached per ``slot`` (a
        stable id: the param-group index and bucket ordinal, never a per-step value) and rebuilt
        only when a pointer or flag in it changes -- so the cache holds at most one table per
        slot and a replaced state buffer can never leave a stale pointer behind."""
        key = tuple((r[0].data_ptr(), r[1].data_ptr(), r[2].data_ptr() if r[2] is not None else 0,
                     r[3].data_ptr() if r[3] is not None else 0, r[4].data_ptr() if r[4] is not None else 0,
                     r[5], r[0].numel(), r[1].dtype,
                     tuple(t.data_ptr() for t in r[6]) if len(r) > 6 and r[6] is not None else ()) for r in rows)
        cache = self._tables
        if cache.get(slot, (None,))[0] != key:
            cache[slot] = (key, build_table(rows, rows[0][0].device))
        meta, nt, nb = cache[slot][1]
        ops().fused_opt_step(meta, nt, nb, self._mode, *hp)
        bump_write_generation()


class FusedSGD(_FusedMixin, SGD):
    _mode = MODE_SGD

    def __init__(self, params, **kw):
        super().__init__(params, **kw)
        self._fused_init()

    @torch.no_grad()
    def step(self, closure=None):
        if not all(self._can_fuse(g) for g in self.param_groups if any(p.grad is not None for p in g["params"])):
            self.last_step_fused = False
            return super().step(closure)
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        ema_w = self.ema_weight
        shadows = weight_shadows([p for g in self.param_groups for p in g["params"] if p.grad is not None])
        for gi, group in enumerate(self.param_groups):
            mom = float(group["momentum"])
            rows = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                first = False
                buf = None
                if mom != 0.0:
                    buf = st.get("momentum_buffer")
                    if buf is None:
                        buf = st["momentum_buffer"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                        first = True
                    elif not same_layout(buf, p):  # e.g. loaded from a checkpoint in another layout
                        buf = st["momentum_buffer"] = torch.empty_like(p).copy_(buf)
                rows.append((p, p.grad, buf, None, self._ema_of.get(p) if ema_w is not None else None, first,
                             shadows.get(p)))
            if not rows:
                continue
            lr = float(group["lr"])
            hp = (lr, mom, float(group["dampening"]), float(group["weight_decay"]), bool(group["nesterov"]),
                  0.0, 0.0, 0.0, 0.0, 0.0, 1.0, float(ema_w) if ema_w is not None else 0.0)
            self._launch(gi, rows, hp)
        self._crsk(shadows)
        shadows_written(shadows)
        self.last_step_fused = ema_w is not None and bool(self._ema_of)
        self.fused_steps += 1
        return loss


class _FusedAdamBase(_FusedMixin):
    @torch.no_grad()
    def step(self, closure=None):
        if not all(self._can_fuse(g) for g in self.param_groups if any(p.grad is not None for p in g["params"])):
            self.last_step_fused = False
            return super().step(closure)
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        ema_w = self.ema_weight
        shadows = weight_shadows([p for g in self.param_groups for p in g["params"] if p.grad is not None])
        for gi, group in enumerate(self.param_groups):
            beta1, beta2 = (float(b) for b in group["betas"])
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                for k in ("exp_avg", "exp_avg_sq"):  # checkpoint-loaded state may be in another layout
                    if not same_layout(st[k], p):
                        st[k] = torch.empty_like(p).copy_(st[k])
                st["step"] += 1
                by_step.setdefault(float(st["step"]), []).append(
                    (p, p.grad, st["exp_avg"], st["exp_avg_sq"],
                     self._ema_of.get(p) if ema_w is not None else None, False, shadows.get(p)))
            lr = float(group["lr"])
            # normally one bucket; several only after loading a hand-assembled state
            for bi, (steps, rows) in enumerate(sorted(by_step.items())):
                bc1 = 1.0 - beta1 ** steps
                bc2 = 1.0 - beta2 ** steps
                hp = (lr, 0.0, 0.0, float(group["weight_decay"]), False, beta1, beta2, float(group["eps"]),
                      lr / bc1, 1.0 / math.sqrt(bc2), 1.0, float(ema_w) if ema_w is not None else 0.0)
                self._launch((gi, bi), rows, hp)
        self._crsk(shadows)
        shadows_written(shadows)
        self.last_step_fused = ema_w is not None and bool(self._ema_of)
        self.fused_steps += 1
        return loss


class FusedAdam(_FusedAdamBase, Adam):
    _mode = MODE_ADAM

    def __init__(self, params, **kw):
        super().__init__(params, **kw)
        self._fused_init()


class FusedAdamW(_FusedAdamBase, AdamW):
    _mode = MODE_ADAMW

    def __init__(self, params, **kw):
        super().__init__(params, **kw)
        self._fused_init()


_EMA_TABLES: dict = {}


def ema_lerp_(pairs, weight: float):
    """e <- lerp(e, src, weight) over [(src, e)] fp32 CUDA tensors in one launch (BN running stats)."""
    rows = [(s, s, None, None, e, False) for s, e in pairs]
    if not rows:
        return
    # sizes too: a later set of tensors may reuse the same addresses with other shapes
    key = tuple((r[0].data_ptr(), r[4].data_ptr(), r[0].numel()) for r in rows)
    tab = _EMA_TABLES.get(key)
    if tab is None:
        if len(_EMA_TABLES) > 16:
            _EMA_TABLES.clear()
        tab = _EMA_TABLES[key] = build_table(rows, rows[0][0].device)
    meta, nt, nb = tab
    ops().ema_lerp(meta, nt, nb, float(weight))
    bump_write_generation()
