"""Dense convolution on the hand-written MFMA kernels (``csrc/kernels/conv_igemm.hip``, and the
older 16x16x32 ``conv_mfma.hip`` for Cin % 64 != 0).

Reference: the ``nn.Conv2d`` of every ConvBNAct / residual block (models/modules.py:73-85,
ddrnet.py:168-219), executed by cuDNN in the reference (forward, backward-data and
backward-filter) and followed by a separate BatchNorm pass.  Here, for channels-last bf16
activations, every such conv is ONE autograd node (:class:`_ConvFn`) whose three passes are
each routed to our kernel or to MIOpen:

* forward (training): ``conv_igemm`` with the BN statistics in its epilogue (per-channel sum /
  sum of squares -> a [G, 2C] slab that ``ops.bn_act`` finalizes), so the BatchNorm forward no
  longer re-reads the conv output;
* data gradient: ``conv_igemm_dgrad`` -- the same gather kernel over dy with a flipped tap
  table (one launch per output phase for strided convs, no col2im, no zero-fill);
* stride-1 3 x 3 convs (forward and data gradient) also have the
  halo-tiled kernel ``conv_halo`` (``csrc/kernels/conv_halo.hip``): the input tile + halo of a
  64-channel chunk is staged in LDS once and every tap reads a shifted window of it, instead of
  re-gathering each pixel once per tap;
* 3 x 3 stride-1 convs that sum over exactly 64 channels (forward Cin = 64, data gradient of
  Cout = 64 -- DDRNet's layer1 at 256 x 512) also have ``conv_wres`` (``csrc/kernels/conv_wres.hip``):
  the block's whole 64 x 9 x 64 weight slice stays in LDS and only the input halo streams;
* weight gradient: ``conv_igemm_wgrad`` -- split-K over pixels with transposed LDS reads, fp32
  partial tiles reduced deterministically straight into the fp32 weight-gradient layout
  (MIOpen's wrw needs a zero-filled output buffer every call);
* inference: ``conv_igemm`` with BatchNorm (running statistics), residual add and ReLU / ReLU6
  folded into the epilogue -- one kernel per ConvBNAct / RB tail.

Each pass of each layer shape is timed once against MIOpen the first time it runs
(``cudnn.benchmark``-style; never during HIP-graph capture) and the faster one is kept --
``decisions()`` lists the outcomes.  ``RTSEG_CONV_MFMA=0`` disables our kernels, ``=1`` forces
them wherever they apply; ``RTSEG_CONV_HALO=0`` drops the halo kernel from the candidates,
``=1`` puts it first (so ``RTSEG_CONV_MFMA=1`` forces it where it applies); ``RTSEG_CONV_WRES``
likewise for ``conv_wres``.
"""
from __future__ import annotations

import os
import weakref

from typing import NamedTuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import ops, use_hip, write_generation
from .dilated import PrunedConv2d, has_dead_taps, pruned_conv2d

_DECISIONS: dict = {}

# Persistent tuning database: per-shape winners of earlier runs on this GPU architecture, so a
# fresh process skips the timing (a 1024x2048 DDRNet-23 step tunes ~70 pass shapes).  Read from
# RTSEG_TUNE_DB (default: the in-tree miopen_db/rtseg_conv_decisions.json, next to MIOpen's find
# database); new decisions are written to RTSEG_TUNE_DB_OUT when set.  RTSEG_TUNE_DB=none: off.
_DB_DEFAULT = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                           "miopen_db", "rtseg_conv_decisions.json")
_DB = None


def _arch() -> str:
    try:
        return torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName.split(":")[0]
    except Exception:  # noqa: BLE001 - no device: nothing to look up
        return ""


def _tune_db() -> dict:
    global _DB
    if _DB is None:
        _DB = {}
        path = os.environ.get("RTSEG_TUNE_DB", _DB_DEFAULT)
        if path != "none" and os.path.isfile(path):
            import json

            try:
                with open(path) as f:
                    data = json.load(f)
                if data.get("arch") == _arch():
                    _DB = dict(data.get("decisions", {}))
            except (OSError, ValueError):
                _DB = {}
    return _DB


def _db_record(key, name):
    """Add one decision to RTSEG_TUNE_DB_OUT: merged with what the file already holds (other
    processes' or earlier runs' entries survive), written atomically, by global rank 0 only
    (every DDP rank times the same shapes)."""
    db = _tune_db()
    db[repr(key)] = name
    out = os.environ.get("RTSEG_TUNE_DB_OUT")
    if not out or os.environ.get("RANK", "0") != "0":
        return
    import json

    merged = {}
    if os.path.isfile(out):
        try:
            with open(out) as f:
                data = json.load(f)
            if data.get("arch") == _arch():
                merged = dict(data.get("decisions", {}))
        except (OSError, ValueError):
            merged = {}
    merged.update(db)
    tmp = f"{out}.{os.getpid()}.tmp"
    with open(tmp, "w") as f:
        json.dump({"arch": _arch(), "decisions": dict(sorted(merged.items()))}, f, indent=0)
    os.replace(tmp, out)


def _mode() -> str:
    return os.environ.get("RTSEG_CONV_MFMA", "auto")


def _halo_mode() -> str:
    return os.environ.get("RTSEG_CONV_HALO", "auto")


def halo_ok(conv, reduce_c: int, out_c: int) -> bool:
    """Shapes ``conv_halo`` takes: 3 x 3, stride 1, dilation 1, 64-channel multiples on both
    sides (``reduce_c``: channels summed over, ``out_c``: produced)."""
    if _halo_mode() == "0" or tuple(conv.stride) != (1, 1):
        return False
    if tuple(conv.kernel_size) != (3, 3) or tuple(conv.dilation) != (1, 1):
        return False
    return reduce_c % 64 == 0 and out_c % 64 == 0 and max(reduce_c, out_c) <= 8192


def _npix(x: torch.Tensor) -> int:
    return x.shape[0] * x.shape[2] * x.shape[3]


def _fits32(npix: int, c: int) -> bool:
    """The halo-staging kernels address the summed-over tensor with 32-bit buffer offsets."""
    return npix * c * 2 < (1 << 31)


def wres_ok(conv, reduce_c: int, out_c: int, npix: int) -> bool:
    """Shapes ``conv_wres`` takes (``csrc/kernels/conv_wres.hip``): 3 x 3, stride 1, pad 1,
    dilation 1, exactly 64 channels summed over, a multiple of 64 produced, < 2 GB summed over
    (``npix`` = N * H * W)."""
    if os.environ.get("RTSEG_CONV_WRES", "auto") == "0":
        return False
    return (tuple(conv.kernel_size) == (3, 3) and tuple(conv.stride) == (1, 1) and tuple(conv.padding) == (1, 1)
            and tuple(conv.dilation) == (1, 1) and reduce_c == 64 and out_c % 64 == 0
            and _fits32(npix, reduce_c))


# the 8-wave 1 x 4-tile conv_hreg layout as an autotune candidate (RTSEG_CONV_HREG4=0: off, A/B)
_HREG4 = os.environ.get("RTSEG_CONV_HREG4", "1") != "0"
# ... and the same layout with double-buffered accumulators: the epilogue of tile t drained beside
# tile t + 1's MFMAs.  Opt-in (RTSEG_CONV_HREG5=1): measured neutral -- 359 vs 355 us (fwd + stats)
# and 346 vs 349 us (dgrad) on the 128-channel layer, headline 566.2-567.0 images/s either way
# (profiles/r6_hreg)
_HREG5 = os.environ.get("RTSEG_CONV_HREG5", "0") == "1"


def hreg_ok(conv, reduce_c: int, out_c: int, npix: int) -> bool:
    """Shapes ``conv_hreg`` takes (``csrc/kernels/conv_hreg.hip``): 3 x 3, stride 1, pad 1, dilation
    1, a 64-channel multiple summed over, a 128-channel multiple produced.  Two candidates: "hreg"
    (8 waves x 1 tile row) and "hreg2" (4 waves x 2 rows: half the weight stream)."""
    if os.environ.get("RTSEG_CONV_HREG", "auto") == "0":
        return False
    return (tuple(conv.kernel_size) == (3, 3) and tuple(conv.stride) == (1, 1) and tuple(conv.padding) == (1, 1)
            and tuple(conv.dilation) == (1, 1) and reduce_c % 64 == 0 and out_c % 128 == 0
            and _fits32(npix, reduce_c))


def whalo_ok(conv, cin: int, cout: int, npix: int) -> bool:
    """Weight gradients ``conv_whalo_wgrad`` takes (``csrc/kernels/conv_whalo.hip``): 3 x 3,
    stride 1, pad 1, dilation 1, 64-channel multiples on both sides."""
    if os.environ.get("RTSEG_CONV_WHALO", "auto") == "0":
        return False
    return (tuple(conv.kernel_size) == (3, 3) and tuple(conv.stride) == (1, 1) and tuple(conv.padding) == (1, 1)
            and tuple(conv.dilation) == (1, 1) and cin % 64 == 0 and cout % 64 == 0
            and _fits32(npix, max(cin, cout)))


# RTSEG_CONV_STEM=0 / RTSEG_TWIN_CONV=0: A/B switches (bench 486.8 -> 490.9 images/s with both on,
# profiles/r4_stem)
_STEM_DEFAULT = "auto"
_TWIN_DEFAULT = "1"


def stem_ok(conv, x: torch.Tensor) -> bool:
    """Convs ``conv_stem`` takes (``csrc/kernels/conv_stem.hip``): 3 input channels, 3 x 3, pad 1,
    dilation 1, stride 1 or 2, a multiple of 16 up to 64 produced, even input width."""
    if os.environ.get("RTSEG_CONV_STEM", _STEM_DEFAULT) == "0":
        return False
    return (conv.in_channels == 3 and tuple(conv.kernel_size) == (3, 3) and tuple(conv.padding) == (1, 1)
            and tuple(conv.dilation) == (1, 1) and tuple(conv.stride) in ((1, 1), (2, 2))
            and conv.out_channels % 16 == 0 and conv.out_channels <= 64 and x.shape[3] % 2 == 0)


def _order(cands):
    """``RTSEG_CONV_HALO=1`` / ``RTSEG_CONV_WRES=1``: that candidate first (what
    ``RTSEG_CONV_MFMA=1`` forces)."""
    if _halo_mode() == "1":
        cands.sort(key=lambda c: c[0] != "halo" and not c[0].startswith("halo"))
    if os.environ.get("RTSEG_CONV_WRES") == "1":
        cands.sort(key=lambda c: c[0] != "wres")
    if os.environ.get("RTSEG_CONV_WHALO") == "1":
        cands.sort(key=lambda c: c[0] != "whalo")
    if os.environ.get("RTSEG_CONV_WHALO") == "2":
        cands.sort(key=lambda c: c[0] != "whalo2")
    if os.environ.get("RTSEG_CONV_HREG") == "1":
        cands.sort(key=lambda c: c[0] != "hreg")
    if os.environ.get("RTSEG_CONV_HREG") == "2":
        cands.sort(key=lambda c: c[0] != "hreg2")
    if os.environ.get("RTSEG_CONV_HREG") == "4":
        cands.sort(key=lambda c: c[0] != "hreg4")
    if os.environ.get("RTSEG_CONV_HREG") == "5":
        cands.sort(key=lambda c: c[0] != "hreg5")
    if os.environ.get("RTSEG_CONV_STEM") == "1":
        cands.sort(key=lambda c: c[0] != "stem")
    if os.environ.get("RTSEG_CONV_GEMM") == "1":
        cands.sort(key=lambda c: c[0] != "gemm")
    return cands


# ----------------------------------------------------------------------------- pointwise GEMMs
def gemm_ok(conv) -> bool:
    """1 x 1, no padding, stride 1 or 2, ungrouped: each pass is one plain GEMM over the
    channels-last pixel rows (hipBLASLt).  This is the candidate for the pointwise passes the
    implicit-GEMM kernels lose to MIOpen: DDRNet-23's DAPPM 1024 -> 256 at 2 x 4 to 16 x 32, the
    compression 1 x 1s, and the strided 1 x 1 shortcuts' data / weight gradients.
    ``RTSEG_CONV_GEMM=0``: off; ``=1``: first (forced)."""
    return (os.environ.get("RTSEG_CONV_GEMM") != "0" and tuple(conv.kernel_size) == (1, 1)
            and tuple(conv.padding) == (0, 0) and tuple(conv.dilation) == (1, 1)
            and getattr(conv, "groups", 1) == 1 and tuple(conv.stride) in ((1, 1), (2, 2)))


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N*H*W, C] view of a channels-last NCHW tensor (a copy if it is not channels-last dense)."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _subsample(x: torch.Tensor, s: int) -> torch.Tensor:
    """The pixels a stride-s 1 x 1 conv reads (pad 0: rows and columns 0, s, 2s, ...)."""
    return x if s == 1 else x[:, :, ::s, ::s].contiguous(memory_format=torch.channels_last)


def _from_rows(r: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    return r.view(n, h, w, r.shape[1]).permute(0, 3, 1, 2)


def gemm_fwd(x: torch.Tensor, wk: torch.Tensor, s: int) -> torch.Tensor:
    """y = x W^T per pixel: [P, Cin] x [Cin, Cout], the output rows are y's channels-last memory."""
    xs = _subsample(x, s)
    y = torch.mm(_rows(xs), wk.reshape(wk.shape[0], -1).t())
    return _from_rows(y, xs.shape[0], xs.shape[2], xs.shape[3])


def gemm_dgrad(dy: torch.Tensor, wk: torch.Tensor, x_shape, s: int, addend=None) -> torch.Tensor:
    """dx = dy W per output pixel, scattered to the rows / columns the stride read (the rest
    stay zero, or the addend's): one addmm when s == 1."""
    wm = wk.reshape(wk.shape[0], -1)  # [Cout, Cin]
    n, cin, h, w = x_shape
    if s == 1:
        r = torch.mm(_rows(dy), wm) if addend is None else torch.addmm(_rows(addend), _rows(dy), wm)
        return _from_rows(r, n, h, w)
    sub = _from_rows(torch.mm(_rows(dy), wm), n, dy.shape[2], dy.shape[3])
    if addend is None:
        dx = torch.zeros((n, cin, h, w), dtype=dy.dtype, device=dy.device).contiguous(memory_format=torch.channels_last)
        dx[:, :, ::s, ::s] = sub
    else:
        dx = addend.clone(memory_format=torch.channels_last)
        dx[:, :, ::s, ::s] += sub
    return dx


def gemm_wgrad(x: torch.Tensor, dy: torch.Tensor, s: int) -> torch.Tensor:
    """dW = dy^T x over the pixels the stride read: [Cout, P] x [P, Cin], fp32 out."""
    a, b = _rows(dy).t(), _rows(_subsample(x, s))
    try:
        dw = torch.mm(a, b, out_dtype=torch.float32)  # fp32 accumulator written as is
    except (RuntimeError, TypeError):
        dw = torch.mm(a, b).float()
    return dw.view(dw.shape[0], dw.shape[1], 1, 1)


def _autocast_bf16(x: torch.Tensor) -> bool:
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
    return dt == torch.bfloat16


_ROUTED = (nn.Conv2d, PrunedConv2d)


def conv_ok(x: torch.Tensor, conv: nn.Module) -> bool:
    """Convs this module routes (anything else stays ``conv(x)`` on MIOpen): dense, bias-free,
    channels-last bf16 activations.  Which kernel runs each pass is decided per shape."""
    if type(conv) not in _ROUTED or conv.groups != 1 or conv.bias is not None:
        return False
    if conv.padding_mode != "zeros" or isinstance(conv.padding, str):
        return False
    if x.dim() != 4 or not x.is_cuda or _mode() == "0" or not use_hip(x, "conv"):
        return False
    if has_dead_taps(x.shape[2:], conv.kernel_size, conv.stride, conv.padding, conv.dilation):
        return False  # the module's own forward drops the dead taps (ops/dilated.py)
    if conv.kernel_size[0] * conv.kernel_size[1] > 49:
        return False
    return _autocast_bf16(x) and x.is_contiguous(memory_format=torch.channels_last)


def _geom(conv):
    return list(conv.stride), list(conv.padding), list(conv.dilation)


def _cached(conv, attr, make):
    """bf16 re-layouts of the fp32 weight.  Cached on the module only for inference (no grad /
    eval): in training the fused optimizer rewrites parameters through raw pointers, which does
    not bump their version counters, so a cached copy could go stale -- the training path
    builds the copy once per forward and hands it to its backward instead."""
    w = conv.weight
    if conv.training and torch.is_grad_enabled():
        return make(w.detach())
    key = (w.data_ptr(), w._version, write_generation())
    hit = getattr(conv, attr, None)
    if hit is not None and hit[0] == key:
        return hit[1]
    t = make(w.detach())
    setattr(conv, attr, (key, t))
    return t


class _Shadow:
    """bf16 copies of a trained conv weight in the two layouts the kernels read -- krsc [Cout, KH,
    KW, Cin] (forward) and crsk [Cin, KH, KW, Cout] (data gradient) -- rewritten by the fused
    optimizer step itself (ops/optim.py passes them to optim.hip), so a training step has no
    per-conv cast and transpose kernels (~100 launches per DDRNet-23 step).  Valid while the
    weight is what the last fused step (or the last refresh) left: same storage, same version
    counter (any other in-place write bumps it) and the same optimizer generation."""

    __slots__ = ("krsc", "crsk", "gen", "crsk_gen", "version", "ptr")

    def __init__(self, w):
        cout, cin, kh, kw = w.shape
        self.krsc = torch.empty((cout, kh, kw, cin), dtype=torch.bfloat16, device=w.device)
        self.crsk = torch.empty((cin, kh, kw, cout), dtype=torch.bfloat16, device=w.device)
        self.gen = self.crsk_gen = -1
        self.version = self.ptr = None


_OPT_GEN = [0]  # fused optimizer steps that rewrote the shadows
_SHADOW_ON = os.environ.get("RTSEG_WEIGHT_SHADOW", "1") != "0"  # A/B: per-step cast + transpose


def _shadow_current(w, sh, crsk=False) -> bool:
    return ((sh.crsk_gen if crsk else sh.gen) == _OPT_GEN[0] and sh.version == w._version
            and sh.ptr == w.data_ptr())


def shadow_of(w):
    """The :class:`_Shadow` of a conv weight (an attribute of the Parameter: a tensor cannot key a
    weak dict -- its ``==`` is elementwise), or None."""
    return getattr(w, "_rtseg_shadow", None)


def weight_shadows(params):
    """{param: (krsc, crsk)} of the shadowed conv weights among ``params`` (for the fused step)."""
    return {p: (sh.krsc, sh.crsk) for p in params if (sh := shadow_of(p)) is not None}


def shadows_written(params) -> None:
    """The fused step just rewrote these parameters' shadows (ops/optim.py, after its launch)."""
    _OPT_GEN[0] += 1
    for p in params:
        sh = shadow_of(p)
        if sh is not None:
            sh.gen = sh.crsk_gen = _OPT_GEN[0]
            sh.version, sh.ptr = p._version, p.data_ptr()


def invalidate_weight_shadows(params) -> int:
    """Mark the bf16 shadows of ``params`` stale (rebuilt from the fp32 weight on next use).  For
    parameter writes the shadow's validity key cannot see: a write through ``p.data`` (a
    separate version counter), a collective into the parameter storage (DDP's initial broadcast,
    ``parallel/ddp.py`` calls this), raw-pointer writers other than the fused step.  Writes
    through ``p`` itself under ``torch.no_grad()`` (``load_state_dict``, ``p.copy_``) bump the
    version counter and need no call.  Returns the number of shadows invalidated."""
    from ._ext import bump_write_generation

    bump_write_generation()  # every (ptr, version, generation)-keyed cache: depth-wise, eval BN, w16
    n = 0
    for p in params:
        if getattr(p, "_rtseg_dw_wt", None) is not None:
            p._rtseg_dw_wt = None  # the depth-wise kernels' fp32 weight re-layout (ops/dwconv.py)
        sh = shadow_of(p)
        if sh is not None:
            sh.gen = sh.crsk_gen = -1
            sh.version = sh.ptr = None
            n += 1
    return n


def _train_shadow(conv, crsk=False) -> torch.Tensor:
    w = conv.weight
    sh = shadow_of(w)
    if sh is None or sh.krsc.shape != (w.shape[0], w.shape[2], w.shape[3], w.shape[1]) or sh.krsc.device != w.device:
        sh = w._rtseg_shadow = _Shadow(w)
    if not _shadow_current(w, sh, crsk):
        if (sh.version, sh.ptr) != (w._version, w.data_ptr()) or sh.gen != _OPT_GEN[0]:
            sh.gen = sh.crsk_gen = -1  # a write the optimizer did not make: both layouts are stale
        with torch.no_grad():
            if crsk:
                sh.crsk.copy_(w.detach().permute(1, 2, 3, 0))
            else:
                sh.krsc.copy_(w.detach().permute(0, 2, 3, 1))
        if crsk:
            sh.crsk_gen = _OPT_GEN[0]
        else:
            sh.gen = _OPT_GEN[0]
        sh.version, sh.ptr = w._version, w.data_ptr()
    return sh.crsk if crsk else sh.krsc


def weight_krsc(conv: nn.Conv2d) -> torch.Tensor:
    """[Cout, KH, KW, Cin] bf16 (forward B operand).  Training: the fused optimizer's shadow."""
    w = conv.weight
    if getattr(conv, "_rtseg_dense_view", False):  # a per-call block-diagonal weight: never cached
        return w.detach().to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
    # (called inside _ConvFn.forward, where autograd is off: a trainable weight of a module in
    # training mode is the test)
    if _SHADOW_ON and conv.training and w.requires_grad and w.is_cuda and w.dtype == torch.float32:
        return _train_shadow(conv)
    return _cached(conv, "_rtseg_wk", lambda w: w.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous())


def weight_crsk(conv: nn.Conv2d, wk: torch.Tensor) -> torch.Tensor:
    """[Cin, KH, KW, Cout] bf16 (data-gradient B operand) for the ``wk`` this conv's forward used."""
    sh = shadow_of(conv.weight)
    if sh is not None and wk is sh.krsc:
        return _train_shadow(conv, crsk=True)
    return wk.permute(3, 1, 2, 0).contiguous()


def _time(fn, reps=8, warm=True):
    """GPU time of ``fn`` (eager; the candidates are >= tens of microseconds at training sizes)."""
    if warm:
        fn()
        torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e)


def _wall_ms(fn) -> float:
    """Wall-clock milliseconds of one synchronised call (includes any host-side work: MIOpen's
    find / kernel compilation on a shape it has no record of)."""
    import time

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


# A vendor candidate whose first (warm) call takes longer than this many ms AND this many times
# the best native candidate's time is dropped without further calls (RTSEG_TUNE_BUDGET_MS).
_VENDOR_BUDGET_MS = float(os.environ.get("RTSEG_TUNE_BUDGET_MS", "50"))
_VENDOR_BUDGET_X = 25.0


def _choose(key, candidates):
    """Index of the fastest candidate (timed once per key, never while a graph is captured).
    ``candidates``: [(name, fn)] with ours first and MIOpen ("miopen") last; ``RTSEG_CONV_MFMA=1``
    forces index 0.

    Bounded first-step cost at a new shape: the native candidates are timed first (one warm and
    one timed call each); MIOpen's warm call is then clocked on the wall, and if it exceeded both
    ``_VENDOR_BUDGET_MS`` and ``_VENDOR_BUDGET_X`` x the best native time (an immediate-mode
    fallback to a naive kernel, or a find-mode search) it is dropped with no further call.  The
    survivors within 4x of the best get three interleaved rounds, best of each, so one noisy round
    (clock ramp, a neighbour's allocation) cannot flip the pick."""
    if len(candidates) == 1 or _mode() == "1":
        return 0
    names = [n for n, _ in candidates]
    if os.environ.get("RTSEG_TUNE_FIXED") == "1":
        # reproducible across processes (numerics tests): the first native candidate, never a
        # timing -- nor a decision an earlier timing in this process made
        return next((i for i, n in enumerate(names) if n != "miopen"), 0)
    got = _DECISIONS.get(key)
    if got is not None:  # by name: the candidate list may differ (e.g. RTSEG_CONV_HALO changed)
        if got[1] in names:
            return names.index(got[1])
    saved = _db_pick(_tune_db().get(repr(key)), names)
    if saved is not None:  # an earlier run's winner for this shape (persistent tuning database)
        _DECISIONS[key] = (names.index(saved), saved, [])
        return names.index(saved)
    if os.environ.get("RTSEG_DETERMINISTIC") == "1":
        # config.deterministic (utils/runtime.py): a shape the database lacks takes the first
        # native candidate instead of a timing, so every process runs the same kernels
        fixed = next((i for i, n in enumerate(names) if n != "miopen"), 0)
        _DECISIONS[key] = (fixed, names[fixed], [])
        return fixed
    if torch.cuda.is_current_stream_capturing():
        return len(candidates) - 1  # MIOpen is last
    with torch.no_grad():
        native = [i for i, n in enumerate(names) if n != "miopen"]
        first = {i: _time(candidates[i][1], reps=1) for i in native}
        best_native = min(first.values()) if first else float("inf")
        dropped = set()
        for i in range(len(candidates)):
            if i in first:
                continue
            wall = _wall_ms(candidates[i][1])
            if native and wall > max(_VENDOR_BUDGET_MS, _VENDOR_BUDGET_X * best_native):
                first[i] = wall
                dropped.add(i)
                continue
            first[i] = _time(candidates[i][1], reps=1, warm=False)
        lo = min(first.values())
        live = [i for i in range(len(candidates)) if i not in dropped and first[i] <= 4 * lo]
        rounds = [{i: _time(candidates[i][1], reps=4, warm=False) / 4 for i in live} for _ in range(3)]
        times = [min(r[i] for r in rounds) if i in live else first[i] for i in range(len(candidates))]
    best = min(range(len(times)), key=times.__getitem__)
    _DECISIONS[key] = (best, candidates[best][0], [round(t, 4) for t in times])
    _db_record(key, candidates[best][0] + "@" + "+".join(sorted(names)))
    return best


# candidates of the round-3 tuning database, whose entries are bare winner names
_LEGACY_CANDS = {"igemm", "igemm_nostats", "halo", "mfma", "miopen"}


def _db_pick(entry, names):
    """The tuning-database winner for a candidate list, or None: an entry ``winner@c1+c2+...``
    counts only for the same candidate set (a new kernel family re-times the shapes it applies
    to); a bare legacy entry only when every candidate predates the record format."""
    if not entry:
        return None
    win, _, among = entry.partition("@")
    if among:
        return win if win in names and sorted(among.split("+")) == sorted(names) else None
    return win if win in names and set(names) <= _LEGACY_CANDS else None


# ----------------------------------------------------------------------------- autograd node
def _conv_fwd(x, weight, conv, stats, store=True):
    """(y, BN statistics slab | None, KRSC bf16 weight, autotune key) of a routed conv.
    ``store=False`` (the stem kernel with statistics only): y is allocated, never written."""
    stride, padding, dilation = _geom(conv)
    cout, cin, kh, kw = weight.shape
    key = (tuple(x.shape), cout, kh, kw, tuple(stride), tuple(padding), tuple(dilation))
    part = None
    wk = weight_krsc(conv)
    impl = _fwd_impl(x, wk, conv, key, stats)
    if impl == "igemm":
        y, part = ops().conv_igemm(x, wk, stride, padding, dilation, stats, None, None, 0)
    elif impl == "igemm_nostats":  # short-K convs: the epilogue reduction costs more than a pass
        y, part = ops().conv_igemm(x, wk, stride, padding, dilation, False, None, None, 0)
    elif impl == "halo":
        y, part = ops().conv_halo(x, wk, stride, padding, dilation, stats, None, None, 0)
    elif impl == "wres":
        y, part = ops().conv_wres(x, wk, stride, padding, dilation, stats)
    elif impl in ("hreg", "hreg2", "hreg4", "hreg5"):
        y, part = ops().conv_hreg(x, wk, stride, padding, dilation, stats,
                                  {"hreg2": 2, "hreg4": 4, "hreg5": 5}.get(impl, 1))
    elif impl == "mfma":
        y, part = ops().conv_mfma(x, wk, stride, padding, dilation, stats, None, None, 0)
    elif impl == "stem":
        y, part = ops().conv_stem(x, wk, stride, padding, dilation, stats, store or not stats)
    elif impl == "gemm":
        y = gemm_fwd(x, wk, stride[0])
    else:
        y = F.conv2d(x, wk.permute(0, 3, 1, 2), None, stride, padding, dilation)
        y = y.contiguous(memory_format=torch.channels_last)
    if part is not None and part.numel() == 0:
        part = None
    return y, part, wk, key


# Routed-conv nodes by input tensor (weak on both sides): a later consumer of the same tensor that
# is NOT downstream of the conv (a sibling, e.g. the skip of DDRNet's bilateral-fusion upsample,
# whose other consumer is the fusion's 3 x 3 conv) may hand its gradient to the conv's dgrad
# epilogue -- if, at its backward, the conv node has not run yet (consumer_for / ran flag).
_CONSUMERS = weakref.WeakValueDictionary()  # id(input tensor) -> routed-conv node


def _register_consumer(x: torch.Tensor, node) -> None:
    if x.requires_grad:
        _CONSUMERS[id(x)] = node


def consumer_for(t: torch.Tensor):
    """The routed-conv node registered for exactly this tensor (same object: id and in_key) whose
    backward has not run and whose addend slot is free (see _register_consumer), or None."""
    node = _CONSUMERS.get(id(t))
    if node is None or node.ran or node.addend_slot is not None:
        return None
    if node.in_key != (t.data_ptr(), tuple(t.shape), t.dtype):
        return None
    return node


class _ConvFn(torch.autograd.Function):
    """y (+ BN statistics slab) = conv(x, w); backward via our dgrad / wgrad or MIOpen."""

    @staticmethod
    def forward(ctx, x, weight, conv, stats, store=True):
        # store=False: a stem whose BN recomputes the conv output wherever it needs it (ops/bn.py):
        # the statistics launch writes no 2.1 GB y (honoured only on the stem kernel's fused path)
        stem_fused = (_STEM_BN_FUSE and not x.requires_grad and stem_ok(conv, x)
                      and conv.out_channels in (16, 32, 64))
        store = store or not (stem_fused and stats and _impl_is_stem(x, weight, conv, stats))
        y, part, wk, key = _conv_fwd(x, weight, conv, stats, store)
        ctx.y_stored = store
        ctx.save_for_backward(x, wk)
        ctx.conv, ctx.key = conv, key
        # identity of the input, so a residual-add node downstream can hand this node the
        # residual branch's gradient to fuse into the dgrad epilogue (see ops.bn)
        ctx.in_key = (x.data_ptr(), tuple(x.shape), x.dtype)
        ctx.addend_slot = None
        ctx.ran = not ctx.needs_input_grad[0]  # consumer_for: only a node that will produce dx
        _register_consumer(x, ctx)
        ctx.wdtype = weight.dtype
        # a BN node that produced x: from this node's backward, between dgrad and wgrad, a multi-rank
        # SyncBN issues its all-reduce and a single-GPU BN runs its backward on a side stream
        # (ops.bn.bn_bwd_early)
        prod = x.grad_fn
        ctx.bn_node = prod if getattr(prod, "early", None) is not None else None
        # a 3-channel stem conv on an input that needs no gradient: a following batch-statistics
        # BN may hand its backward over (ops.bn), and the BN's dx pass runs inside this conv's
        # weight gradient (conv_stem_wgrad_bn) instead of writing dx to HBM
        ctx.bn_fuse_slot = [] if stem_fused else None
        # ... and its forward apply recomputes this conv from the image with the BN epilogue
        # (conv_stem_bn_act) instead of re-reading y
        ctx.stem_io = ((x, wk) + tuple(_geom(conv))) if ctx.bn_fuse_slot is not None else None
        if part is not None:
            ctx.mark_non_differentiable(part)
        # the statistics slab never gets a gradient: without this autograd would allocate and
        # zero-fill one [slabs, 2C] tensor per conv per step (~50 fill kernels per DDRNet step)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart):
        ctx.ran = True
        if dy is None:
            if ctx.addend_slot:  # a handed-over gradient is this input's whole gradient now
                return _plain(ctx.addend_slot.pop()), None, None, None, None
            return None, None, None, None, None
        x, wk = ctx.saved_tensors
        fused = ctx.bn_fuse_slot.pop() if ctx.bn_fuse_slot else None
        if fused is not None:
            return None, _stem_wgrad_bn(x, ctx.conv, ctx.wdtype, dy, fused, wk, ctx.y_stored), None, None, None
        addend = ctx.addend_slot.pop() if ctx.addend_slot else None
        node, ctx.bn_node = ctx.bn_node, None
        on_dx = None
        if node is not None:
            from .bn import bn_bwd_early

            def on_dx(dx):
                bn_bwd_early(node, dx)
        dx, dw = _conv_bwd(x, wk, ctx.conv, ctx.key, dy, ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                           ctx.wdtype, addend, on_dx)
        return dx, dw, None, None, None


def _impl_is_stem(x, weight, conv, stats) -> bool:
    """Whether the forward of this stem conv runs on the stem kernel (its autotune decision)."""
    stride, padding, dilation = _geom(conv)
    cout, cin, kh, kw = weight.shape
    key = (tuple(x.shape), cout, kh, kw, tuple(stride), tuple(padding), tuple(dilation))
    return _fwd_impl(x, weight_krsc(conv), conv, key, stats) == "stem"


def stem_store_skippable(x: torch.Tensor, conv: nn.Module, bn: nn.Module) -> bool:
    """A training stem ConvBNAct whose BN (batch statistics, no residual / concat slice, a fused
    activation) will recompute the stem conv's output from the image in forward and backward
    (ops/bn.py): its statistics launch need not store the output (``conv_bn_stats(store=False)``)."""
    from .bn import _STEM_BN_RECOMPUTE

    return (_STEM_NO_STORE and _STEM_BN_RECOMPUTE and _STEM_BN_FUSE and use_hip(x, "conv") and torch.is_grad_enabled()
            and conv.weight.requires_grad and not x.requires_grad and bn.training and not padded_ok(conv)
            and stem_ok(conv, x) and conv.out_channels in (16, 32, 64))


# RTSEG_STEM_NO_STORE=1: the stem's statistics launch stores no output and the fused weight
# gradient recomputes the BN input instead of reading it.  Opt-in: on DDRNet-23 b32 the recompute
# inside the weight gradient cost +0.46 ms against the 0.2 ms the skipped store saves
# (profiles/r5_stemrc); the forward apply and the backward reduction recompute either way
_STEM_NO_STORE = os.environ.get("RTSEG_STEM_NO_STORE", "0") == "1"
# RTSEG_STEM_BN_FUSE=0: the stem's BN backward writes dx as before (A/B, tests)
_STEM_BN_FUSE = os.environ.get("RTSEG_STEM_BN_FUSE", "1") != "0"


def _stem_wgrad_bn(x, conv, wdtype, dy, fused, wk=None, stored=True):
    """Weight gradient of a stem conv whose output went through a batch-statistics BN that handed
    its backward over (``fused`` = (bn output grad, bn input, kcoef, mean_invstd, scale_shift,
    act, dummy, full)): the BN's dx is formed while the kernel stages it.  ``dy`` -- what autograd
    passed this node -- is the BN's zero-stride placeholder when the BN was the conv output's only
    consumer; otherwise the placeholder plus the other consumers' gradients, and then the BN's dx
    is materialised (``full()``) and the plain kernel runs on the sum."""
    g, xb, kc, mi, ss, act, dummy, full = fused
    stride, padding, dilation = _geom(conv)
    w = conv.weight
    cl = w.dim() == 4 and w.is_contiguous(memory_format=torch.channels_last) and not w.is_contiguous()
    if dy is dummy or (dy is not None and dy.dim() == 4 and dy.stride() == (0, 0, 0, 0)):
        # a stats-only stem launch stored no BN input: the kernel recomputes it from the image
        rc = wk if (not stored and wk is not None and wk.dtype == torch.bfloat16) else None
        dw = ops().conv_stem_wgrad_bn(x, g, xb, kc, mi, ss, act, 3, 3, stride, padding, dilation, cl, rc)
    else:
        d = full() + dy.to(g.dtype)
        d = d.contiguous(memory_format=torch.channels_last)
        dw = ops().conv_stem_wgrad(x, d, 3, 3, stride, padding, dilation, cl)
    return like_param(dw.to(wdtype), w)


class MaskedAddend(NamedTuple):
    """A residual branch's gradient ``g * act'(z)`` handed to the dgrad of the conv whose input
    is the residual (ops/bn.py) WITHOUT being written out: the BN output's gradient ``g`` and the
    BN's 1-bit activation mask (kMaskBits: element e in bit e % 8 of byte e / 8, channels-last
    order).  The routed dgrad kernels apply the mask in their addend epilogue
    (``addend_mask``); other implementations take :meth:`materialize`."""
    g: torch.Tensor
    bits: torch.Tensor

    def materialize(self) -> torch.Tensor:
        n, c, h, w = self.g.shape
        shifts = torch.arange(8, device=self.bits.device, dtype=torch.uint8)
        m = (self.bits.view(-1, 1) >> shifts) & 1  # [numel / 8, 8] in channels-last element order
        m = m.view(n, h, w, c).permute(0, 3, 1, 2)
        return self.g * m.to(self.g.dtype)


def _plain(addend):
    return addend.materialize() if isinstance(addend, MaskedAddend) else addend


def _conv_bwd(x, wk, conv, key, dy, want_dx, want_dw, wdtype, addend=None, on_dx=None, phase_addend=None):
    """(dx (+ addend) | None, dw | None) of a routed conv.  ``on_dx(dx)`` runs between the data
    and the weight gradient (the early SyncBN all-reduce of the producer BN).  ``phase_addend``:
    added to dx's even rows / columns (see :func:`_dgrad`)."""
    stride, padding, dilation = _geom(conv)
    dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    if dy.data_ptr() % 16:
        dy = dy.clone(memory_format=torch.channels_last)
    dx = dw = None
    if want_dx:
        dx = _dgrad(x, dy, wk, conv, key, stride, padding, dilation, addend, phase_addend)
    elif addend is not None:
        dx = _plain(addend)
    if on_dx is not None and want_dx:
        on_dx(dx)  # dx is the input's whole gradient (a handed-off residual gradient included)
    if want_dw:
        dw = _wgrad(x, dy, wk, conv, key, stride, padding, dilation)
        if dw.dtype != wdtype:
            dw = like_param(dw.to(wdtype), conv.weight)
    return dx, dw


# RTSEG_TWIN_PHASE=0: the twin node's strided 1 x 1 data gradient runs as its own pass (A/B)
_PHASE_FUSE = os.environ.get("RTSEG_TWIN_PHASE", "1") != "0"
PHASE_FUSED = [0]  # twin backward passes that took the phase-addend path (tests)


class _TwinConvFn(torch.autograd.Function):
    """Two routed convs reading the same input -- the 3 x 3 conv and the 1 x 1 projection
    shortcut of a downsampling residual block (DDRNet RB / RBB, reference models/ddrnet.py:168-219)
    -- as ONE autograd node.  Its backward runs once both output gradients exist, so the second
    data gradient takes the first as its epilogue addend: the input gradient is written once,
    with no separate accumulation add of two full-size gradients (autograd's, otherwise)."""

    @staticmethod
    def forward(ctx, x, w1, w2, conv1, conv2):
        y1, p1, wk1, key1 = _conv_fwd(x, w1, conv1, True)
        y2, p2, wk2, key2 = _conv_fwd(x, w2, conv2, True)
        ctx.save_for_backward(x, wk1, wk2)
        ctx.convs, ctx.keys, ctx.wdtypes = (conv1, conv2), (key1, key2), (w1.dtype, w2.dtype)
        ctx.in_key = (x.data_ptr(), tuple(x.shape), x.dtype)  # residual hand-off target (ops.bn)
        ctx.addend_slot = None
        for p in (p1, p2):
            if p is not None:
                ctx.mark_non_differentiable(p)
        ctx.set_materialize_grads(False)
        return y1, p1, y2, p2

    @staticmethod
    def backward(ctx, dy1, _dp1, dy2, _dp2):
        x, wk1, wk2 = ctx.saved_tensors
        want_dx = ctx.needs_input_grad[0]
        dx = ctx.addend_slot.pop() if ctx.addend_slot else None
        dws = [None, None]
        pairs = ((dy1, wk1), (dy2, wk2))
        # the larger-kernel conv last: its data gradient runs on our kernels (whose epilogue adds
        # the other's dx), while a strided 1 x 1 shortcut's often autotunes to MIOpen, where the
        # addend would cost a separate add (profiles/r4_stem)
        order = sorted((0, 1), key=lambda i: ctx.convs[i].kernel_size[0] * ctx.convs[i].kernel_size[1])
        small, big = order
        if (want_dx and dy1 is not None and dy2 is not None and _PHASE_FUSE and gemm_ok(ctx.convs[small])
                and tuple(ctx.convs[small].stride) == (2, 2) and tuple(ctx.convs[big].stride) == (2, 2)
                and ctx.convs[big].in_channels % 8 == 0):
            # the strided 1 x 1 shortcut's data gradient is one GEMM over its output pixels, added
            # by the 3 x 3 conv's dgrad to its even-row / even-column phase: no zero-filled
            # full-size dx, no separate accumulation
            dy_s, wk_s = pairs[small]
            dy_s = dy_s.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            sub = _from_rows(torch.mm(_rows(dy_s), wk_s.reshape(wk_s.shape[0], -1)), x.shape[0], dy_s.shape[2],
                             dy_s.shape[3])
            PHASE_FUSED[0] += 1
            _, dws[small] = _conv_bwd(x, wk_s, ctx.convs[small], ctx.keys[small], dy_s, False,
                                      ctx.needs_input_grad[1 + small], ctx.wdtypes[small])
            dy_b, wk_b = pairs[big]
            dx, dws[big] = _conv_bwd(x, wk_b, ctx.convs[big], ctx.keys[big], dy_b, True, ctx.needs_input_grad[1 + big],
                                     ctx.wdtypes[big], dx, phase_addend=sub)
            return dx, dws[0], dws[1], None, None
        for i in order:
            dy, wk = pairs[i]
            if dy is None:
                continue
            dx, dws[i] = _conv_bwd(x, wk, ctx.convs[i], ctx.keys[i], dy, want_dx, ctx.needs_input_grad[1 + i],
                                   ctx.wdtypes[i], dx)
        return dx if want_dx else None, dws[0], dws[1], None, None


def twin_conv_bn_stats(x: torch.Tensor, conv1: nn.Module, conv2: nn.Module):
    """Training forward of two batch-statistics conv + BN blocks on the same input x (see
    :class:`_TwinConvFn`): ((y1, slab1 | None), (y2, slab2 | None)), or None -> the caller's
    per-conv path (``RTSEG_TWIN_CONV=0``: always)."""
    if os.environ.get("RTSEG_TWIN_CONV", _TWIN_DEFAULT) == "0":
        return None
    if not (conv_ok(x, conv1) and conv_ok(x, conv2)) or padded_ok(conv1) or padded_ok(conv2):
        return None
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    if x.data_ptr() % 16:
        x = x.clone(memory_format=torch.channels_last)
    y1, p1, y2, p2 = _TwinConvFn.apply(x, conv1.weight, conv2.weight, conv1, conv2)
    return (y1, p1), (y2, p2)


def _fwd_impl(x, wk, conv, key, stats) -> str:
    cin, cout = conv.in_channels, conv.out_channels
    stride, padding, dilation = _geom(conv)
    cands = []
    if cin % 64 == 0 and cout % 8 == 0:
        cands.append(("igemm", lambda: ops().conv_igemm(x, wk, stride, padding, dilation, stats, None, None, 0)))
        if stats:
            def nostats():
                y, _ = ops().conv_igemm(x, wk, stride, padding, dilation, False, None, None, 0)
                ops().bn_stats_sums(y)

            cands.append(("igemm_nostats", nostats))
        if halo_ok(conv, cin, cout):
            cands.append(("halo", lambda: ops().conv_halo(x, wk, stride, padding, dilation, stats, None, None, 0)))
        if wres_ok(conv, cin, cout, _npix(x)):
            cands.append(("wres", lambda: ops().conv_wres(x, wk, stride, padding, dilation, stats)))
        if hreg_ok(conv, cin, cout, _npix(x)):
            cands.append(("hreg", lambda: ops().conv_hreg(x, wk, stride, padding, dilation, stats, 1)))
            cands.append(("hreg2", lambda: ops().conv_hreg(x, wk, stride, padding, dilation, stats, 2)))
            if _HREG4:
                cands.append(("hreg4", lambda: ops().conv_hreg(x, wk, stride, padding, dilation, stats, 4)))
            if _HREG5:
                cands.append(("hreg5", lambda: ops().conv_hreg(x, wk, stride, padding, dilation, stats, 5)))
    elif cin % 32 == 0 and cout % 8 == 0:
        cands.append(("mfma", lambda: ops().conv_mfma(x, wk, stride, padding, dilation, stats, None, None, 0)))
    elif stem_ok(conv, x):
        cands.append(("stem", lambda: ops().conv_stem(x, wk, stride, padding, dilation, stats)))
    if gemm_ok(conv):
        def gemm():
            y = gemm_fwd(x, wk, stride[0])
            if stats:
                ops().bn_stats_sums(y)

        cands.append(("gemm", gemm))
    if not cands:
        return "miopen"

    def miopen():
        y = F.conv2d(x, wk.permute(0, 3, 1, 2), None, stride, padding, dilation)
        if stats:
            ops().bn_stats_sums(y)  # the statistics pass our epilogue replaces

    cands.append(("miopen", miopen))
    return cands[_choose(("fwd", stats) + key, _order(cands))][0]


def _dgrad(x, dy, wk, conv, key, stride, padding, dilation, addend=None, phase_addend=None):
    """dx (+ addend: a residual branch's gradient, added in our kernel's epilogue) (+ phase_addend
    on the even rows / columns of a stride-2 dx: a strided 1 x 1 shortcut's data gradient, added
    in the epilogue of the igemm launch of output phase (0, 0))."""
    cin, cout = conv.in_channels, conv.out_channels
    wt = []
    amask = None  # the addend's activation bit mask (MaskedAddend), applied in our epilogues
    if isinstance(addend, MaskedAddend):
        if addend.g.dtype == torch.bfloat16 and addend.g.is_contiguous(memory_format=torch.channels_last) \
                and addend.g.data_ptr() % 16 == 0 and addend.bits.is_contiguous() and cin % 8 == 0:
            addend, amask = addend.g, addend.bits
        else:
            addend = addend.materialize()
    if addend is not None:
        addend = addend.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        if addend.data_ptr() % 16:
            addend = addend.clone(memory_format=torch.channels_last)
    plain = []  # the masked addend written out, for the implementations without a mask epilogue

    def addend_plain():
        if amask is None:
            return addend
        if not plain:
            plain.append(MaskedAddend(addend, amask).materialize())
        return plain[0]

    def ours(fused=False):
        if not wt:  # [Cin, KH, KW, Cout] bf16, the dgrad B operand
            wt.append(weight_crsk(conv, wk))
        return ops().conv_igemm_dgrad(dy, wt[0], list(x.shape), stride, padding, dilation, None, addend, amask,
                                      phase_addend, fused)

    def halo():
        if not wt:
            wt.append(weight_crsk(conv, wk))
        return ops().conv_halo_dgrad(dy, wt[0], list(x.shape), stride, padding, dilation, addend, amask)

    def wres():
        if not wt:
            wt.append(weight_crsk(conv, wk))
        return ops().conv_wres_dgrad(dy, wt[0], list(x.shape), stride, padding, dilation, addend, amask)

    def miopen():  # the addend costs MIOpen a separate add: timed with it
        r = torch.ops.aten.convolution_backward(dy, x, wk.permute(0, 3, 1, 2), None, stride, padding, dilation, False,
                                                [0, 0], 1, [True, False, False])[0]
        return r if addend is None else r + addend_plain()

    def hreg(rows_per_wave=1):
        if not wt:
            wt.append(weight_crsk(conv, wk))
        return ops().conv_hreg_dgrad(dy, wt[0], list(x.shape), stride, padding, dilation, addend, rows_per_wave,
                                     amask)

    cands = [("igemm", ours)] if cout % 64 == 0 and cin % 8 == 0 else []
    if cands and os.environ.get("RTSEG_CONV_DGRAD_PH", "1") != "0" and \
            _fused_phases_ok(x, conv, stride, padding, dilation):  # =0: per-phase launches only (A/B)
        cands.append(("igemm_ph", lambda: ours(True)))
    if halo_ok(conv, cout, cin):
        cands.append(("halo", halo))
    if wres_ok(conv, cout, cin, _npix(x)):
        cands.append(("wres", wres))
    if hreg_ok(conv, cout, cin, _npix(x)):
        cands.append(("hreg", hreg))
        cands.append(("hreg2", lambda: hreg(2)))
        if _HREG4:
            cands.append(("hreg4", lambda: hreg(4)))
        if _HREG5:
            cands.append(("hreg5", lambda: hreg(5)))
    if gemm_ok(conv):
        cands.append(("gemm", lambda: gemm_dgrad(dy, wk, x.shape, stride[0], addend_plain())))
    cands.append(("miopen", miopen))
    # a pass with an addend is its own autotune key: our kernels fuse the add, MIOpen pays for it
    name, fn = cands[_choose(("dgrad",) + key + (("+addend",) if addend is not None else ()), _order(cands))]
    dx = fn()
    if phase_addend is not None and name not in ("igemm", "igemm_ph"):
        dx[:, :, ::stride[0], ::stride[1]] += phase_addend
    return dx


def _fused_phases_ok(x, conv, stride, padding, dilation) -> bool:
    """Whether the igemm data gradient can run every output phase of this strided conv in one
    launch (csrc conv_igemm_dgrad_fused_ok): H, W divisible by the stride, <= 16 phases, and the
    phases' tap tables, padded to the longest, within the kernel's 49 entries."""
    sh, sw = stride
    if sh * sw <= 1 or sh * sw > 16 or x.shape[2] % sh or x.shape[3] % sw:
        return False
    kh, kw = conv.kernel_size
    ph, pw = padding
    dh, dw = dilation
    maxt = max(sum(1 for i in range(kh) for j in range(kw)
                   if (a + ph - i * dh) % sh == 0 and (b + pw - j * dw) % sw == 0)
               for a in range(sh) for b in range(sw))
    return 1 <= maxt and maxt * sh * sw <= 49


def find_conv_consumer(t: torch.Tensor, r: torch.Tensor, max_nodes: int = 64):
    """The routed-conv autograd node (:class:`_ConvFn`) whose input is exactly ``r`` among the
    ancestors of ``t`` -- its backward is then guaranteed to run after the backward of any
    node that consumes ``t`` -- or None."""
    want = (r.data_ptr(), tuple(r.shape), r.dtype)
    seen, stack = set(), [t.grad_fn]
    while stack and len(seen) < max_nodes:
        fn = stack.pop()
        if fn is None or id(fn) in seen:
            continue
        seen.add(id(fn))
        if getattr(fn, "in_key", None) == want:
            return fn
        stack.extend(f for f, _ in fn.next_functions)
    return None


def like_param(g: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
    """``g`` with exactly the strides of parameter ``p``: a free re-stride when both are dense in
    the same memory order (e.g. the (C,1,1,1) vs (C,1,C,C) strides of a 1x1 conv weight), else a
    copy.  The fused optimizer walks param / grad / state linearly in memory and DDP's
    gradient-bucket views want the parameter's strides (no "grad strides do not match bucket
    view strides" copies)."""
    if g.stride() == p.stride():
        return g
    if g.shape == p.shape and _dense(g) and _dense(p):
        big = [i for i in range(g.dim()) if g.shape[i] > 1]
        if sorted(big, key=lambda i: -g.stride(i)) == sorted(big, key=lambda i: -p.stride(i)):
            return g.as_strided(p.shape, p.stride())
    return torch.empty_like(p, dtype=g.dtype).copy_(g)


def _dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense: the size>1 dims tile memory exactly."""
    expected = 1
    for st, sz in sorted((st, sz) for sz, st in zip(t.shape, t.stride()) if sz != 1):
        if st != expected:
            return False
        expected *= sz
    return True


def _wgrad(x, dy, wk, conv, key, stride, padding, dilation):
    cin, cout = conv.in_channels, conv.out_channels
    kh, kw = conv.kernel_size
    w = conv.weight
    cl = w.dim() == 4 and w.is_contiguous(memory_format=torch.channels_last) and not w.is_contiguous()

    def ours():
        return ops().conv_igemm_wgrad(x, dy, kh, kw, stride, padding, dilation, cl or (kh == 1 and kw == 1))

    def whalo(variant=1):
        return ops().conv_whalo_wgrad(x, dy, kh, kw, stride, padding, dilation, cl or (kh == 1 and kw == 1), variant)

    def miopen():
        return torch.ops.aten.convolution_backward(dy, x, wk.permute(0, 3, 1, 2), None, stride, padding, dilation,
                                                   False, [0, 0], 1, [False, True, False])[1]

    def stem():
        return ops().conv_stem_wgrad(x, dy, kh, kw, stride, padding, dilation, cl)

    cands = [("igemm", ours)] if cin % 64 == 0 and cout % 64 == 0 else []
    if whalo_ok(conv, cin, cout, _npix(x)):
        cands.append(("whalo", whalo))
        if os.environ.get("RTSEG_CONV_WHALO2", "1") != "0":
            cands.append(("whalo2", lambda: whalo(2)))  # both output tiles per wave, K split
    if stem_ok(conv, x):
        cands.append(("stem", stem))
    if gemm_ok(conv):
        cands.append(("gemm", lambda: gemm_wgrad(x, dy, stride[0])))
    cands.append(("miopen", miopen))
    cands = _order(cands)
    dw = cands[_choose(("wgrad",) + key, cands)][1]()
    return like_param(dw, w)


# ----------------------------------------------------------------------------- public entry points
def conv_bn_stats(x: torch.Tensor, conv: nn.Conv2d, store: bool = True):
    """Training forward of a conv followed by batch-statistics BN: (y, slab | None).  The slab
    holds the BN statistics of y when our kernel produced y (else ``ops.bn_act`` computes
    them).  None -> the caller's stock path.  ``store=False``: see :func:`stem_store_skippable`."""
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    if x.data_ptr() % 16:
        x = x.clone(memory_format=torch.channels_last)
    return _apply(x, conv, True, store)


# inference: the 128 x 64-tile gather kernel as an autotune candidate (RTSEG_IGEMM_SMALL=0: off)
_SMALL_TILES = os.environ.get("RTSEG_IGEMM_SMALL", "1") != "0"


def conv_bn_act_eval(x: torch.Tensor, conv: nn.Conv2d, bn: nn.Module, act_code: int, residual=None):
    """Inference: act(BN_running(conv(x)) + residual) in one kernel, or None -> caller's path.
    The kernel output has no autograd graph, so a frozen (eval-mode) BN inside a TRAINING step
    -- gradients wanted for x, the conv weight or the residual -- takes the caller's
    differentiable path instead."""
    if bn.training or not bn.track_running_stats or bn.running_mean is None or act_code not in (0, 1, 2):
        return None
    if torch.is_grad_enabled() and (x.requires_grad or conv.weight.requires_grad
                                    or (residual is not None and residual.requires_grad)):
        return None
    if residual is not None and not (residual.is_contiguous(memory_format=torch.channels_last)
                                     and residual.dim() == 4):
        return None
    cin, cout = conv.in_channels, conv.out_channels
    if residual is None and stem7_ok(conv, x):
        return _stem7_eval(x, conv, bn, act_code)
    if (residual is None and conv.bias is None and stem_infer_ok(conv, x) and cout % 16 == 0
            and x.is_cuda and _autocast_bf16(x)):
        # the 3 x 3 stem with the BN + act in its epilogue (one pass; the separate BN apply was
        # 2 % of DDRNet-23's batch-1 inference, profiles/r6_infer)
        from .bn import eval_coeffs

        return _stem_infer(x, conv, None, eval_coeffs(bn)[1], act_code)
    if cout % 8 or cin % 32:
        return None
    x = x.to(torch.bfloat16)
    res = residual.to(torch.bfloat16) if residual is not None else None
    if (x.data_ptr() % 16) or (res is not None and res.data_ptr() % 16):
        return None
    stride, padding, dilation = _geom(conv)
    wk = weight_krsc(conv)
    from .bn import eval_coeffs

    _, ss = eval_coeffs(bn)
    key = ("eval", tuple(x.shape), cout, conv.kernel_size, tuple(stride), tuple(padding), tuple(dilation),
           res is not None)
    op = ops().conv_igemm if cin % 64 == 0 else ops().conv_mfma

    def ours():
        return op(x, wk, stride, padding, dilation, False, ss, res, act_code)[0]

    def small(split_k=False):  # 128 x 64 tiles, 2 blocks per CU: batch-1 layers 256-pixel tiles under-fill
        return ops().conv_igemm_small(x, wk, stride, padding, dilation, ss, res, act_code, split_k)

    def theirs():
        y = F.conv2d(x, wk.permute(0, 3, 1, 2), None, stride, padding, dilation)
        ops().bn_apply(y, ss, res, act_code)

    cands = [("igemm" if cin % 64 == 0 else "mfma", ours)]
    if wres_ok(conv, cin, cout, _npix(x)):  # 64-channel 3 x 3: weights resident in LDS
        cands.append(("wres", lambda: ops().conv_wres_eval(x, wk, stride, padding, dilation, ss, res, act_code)))
    if cin % 64 == 0 and _SMALL_TILES:
        cands.append(("igemm_s", small))
        # ... split over K when even the small tiles leave CUs idle (fp32 parts + one BN pass)
        npix = x.shape[0] * (-(-x.shape[2] // stride[0])) * (-(-x.shape[3] // stride[1]))
        if -(-npix // 128) * -(-cout // 64) < 256:
            cands.append(("igemm_k", lambda: small(True)))
    cands.append(("miopen", theirs))
    pick = _choose(key, cands)
    if cands[pick][0] == "miopen":
        return None
    return cands[pick][1]()


def stem7_ok(conv: nn.Module, x: torch.Tensor) -> bool:
    """A torchvision-style 7 x 7 / pad 3 / stride 2 (or 1) stem on 3 channels with <= 64 (% 16)
    outputs and an even width: ``conv_stem7.hip`` (``RTSEG_CONV_STEM7=0``: off)."""
    return (conv.in_channels == 3 and conv.groups == 1 and tuple(conv.kernel_size) == (7, 7)
            and tuple(conv.padding) == (3, 3) and tuple(conv.dilation) == (1, 1)
            and tuple(conv.stride) in ((1, 1), (2, 2)) and conv.out_channels % 16 == 0 and conv.out_channels <= 64
            and conv.bias is None and x.dim() == 4 and x.shape[1] == 3 and x.shape[3] % 2 == 0
            and conv.padding_mode == "zeros" and os.environ.get("RTSEG_CONV_STEM7", "1") != "0")


def _stem7_eval(x: torch.Tensor, conv: nn.Module, bn: nn.Module, act_code: int):
    """Inference ``act(BN_running(conv(x)))`` of a 7 x 7 stem in one pass (the BN + act on the
    conv's fp32 accumulators), timed once per shape against MIOpen + the BN apply; None -> the
    caller's path.  The KD teacher's ResNet-101 stem (BASELINE config 5): MIOpen took 1.1 ms per
    batch-16 1024 x 2048 call channels-last, plus a BN pass over its 1 GB output
    (tools/bench_stem7.py, profiles/r6_kd)."""
    from .bn import eval_coeffs

    x = x.to(torch.bfloat16)
    if not x.is_contiguous(memory_format=torch.channels_last) or x.data_ptr() % 16:
        x = x.contiguous(memory_format=torch.channels_last).clone(memory_format=torch.channels_last)
    wk = weight_krsc(conv)
    _, ss = eval_coeffs(bn)
    stride = list(conv.stride)

    def ours():
        return ops().conv_stem7(x, wk, stride, ss, act_code)

    def theirs():
        y = F.conv2d(x, wk.permute(0, 3, 1, 2), None, stride, [3, 3], [1, 1])
        ops().bn_apply(y, ss, None, act_code)

    key = ("eval-stem7", tuple(x.shape), conv.out_channels, tuple(stride), act_code)
    if _choose(key, [("stem7", ours), ("miopen", theirs)]) != 0:
        return None
    return ours()


def stem_infer_ok(conv: nn.Module, x: torch.Tensor) -> bool:
    """A 3-channel 3 x 3 stem conv (pad 1, stride 1 / 2, <= 64 outputs, even W) in bf16 inference:
    MIOpen runs these channels-last as ``naive_conv_ab_nonpacked_fwd_nhwc`` (~0.5 ms per 512 x
    1024 image: 18-30 % of DFANet's / ESPNetv2's / FastSCNN's bf16 inference, profiles/r4_end/infer)."""
    return (conv.in_channels == 3 and conv.groups == 1 and tuple(conv.kernel_size) == (3, 3)
            and tuple(conv.padding) == (1, 1) and tuple(conv.dilation) == (1, 1)
            and tuple(conv.stride) in ((1, 1), (2, 2)) and conv.out_channels <= 64 and x.dim() == 4
            and x.shape[1] == 3 and x.shape[3] % 2 == 0 and conv.padding_mode == "zeros"
            and os.environ.get("RTSEG_CONV_STEM", _STEM_DEFAULT) != "0")


def _stem_infer(x: torch.Tensor, conv: nn.Module, bias, bn_ss=None, act_code: int = 0) -> torch.Tensor:
    """``conv(x)`` on ``conv_stem.hip``: the weight zero-padded to the kernel's 16-channel
    granularity (cached, krsc bf16), the real channels sliced back out.  ``bn_ss`` (fp32 [2 Cout],
    Cout % 16 == 0): an eval BN's scale | shift applied with ``act_code`` in the epilogue."""
    cout = conv.out_channels
    cp = -(-cout // 16) * 16

    def make(w):
        w = w.to(torch.bfloat16)
        if cp != cout:
            w = F.pad(w, (0, 0, 0, 0, 0, 0, 0, cp - cout))
        return w.permute(0, 2, 3, 1).contiguous()

    wk = _cached(conv, "_rtseg_stem_wk", make)
    x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    if x.data_ptr() % 16:
        x = x.clone(memory_format=torch.channels_last)
    stride, padding, dilation = _geom(conv)
    if bn_ss is not None:
        return ops().conv_stem_bn_act(x, wk, stride, padding, dilation, bn_ss, act_code)
    if bias is not None:  # added to the fp32 accumulators by the BN epilogue (scale 1): one rounding
        key = (bias.data_ptr(), bias._version, write_generation())
        hit = getattr(conv, "_rtseg_stem_ss", None)
        if hit is None or hit[0] != key:
            ss = torch.zeros(2 * cp, device=x.device, dtype=torch.float32)
            ss[:cp] = 1.0
            ss[cp:cp + cout] = bias.detach().float()
            hit = (key, ss)
            setattr(conv, "_rtseg_stem_ss", hit)
        y = ops().conv_stem_bn_act(x, wk, stride, padding, dilation, hit[1], 0)
    else:
        y, _ = ops().conv_stem(x, wk, stride, padding, dilation, False)
    if cp != cout:
        y = y[:, :cout].contiguous(memory_format=torch.channels_last)
    return y


def conv_forward(x: torch.Tensor, conv: nn.Module) -> torch.Tensor:
    """``conv(x)``; in bf16-autocast inference the bf16 weight copy is cached on the module
    (autocast would re-cast the fp32 weight -- one extra kernel per conv -- every forward), and
    3-channel stem convs run on ``conv_stem.hip`` instead of MIOpen's naive NHWC kernel."""
    if (type(conv) in _ROUTED and not conv.training and not torch.is_grad_enabled() and x.is_cuda
            and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        if stem_infer_ok(conv, x) and use_hip(x, "conv") and _mode() != "0":
            return _stem_infer(x, conv, conv.bias)
        w = conv.weight
        key = (w.data_ptr(), w._version, write_generation(),
               None if conv.bias is None else (conv.bias.data_ptr(), conv.bias._version))
        hit = getattr(conv, "_rtseg_w16", None)
        if hit is None or hit[0] != key:
            b16 = conv.bias.detach().to(torch.bfloat16) if conv.bias is not None else None
            hit = conv._rtseg_w16 = (key, w.detach().to(torch.bfloat16), b16)
        with torch.autocast("cuda", enabled=False):
            return conv._conv_forward(x.to(torch.bfloat16), hit[1], hit[2])
    if conv_ok(x, conv) and torch.is_grad_enabled() and conv.weight.requires_grad:
        y, _ = _apply(x.to(torch.bfloat16), conv, False)
        return y
    if grouped_dense_ok(x, conv):
        return grouped_as_dense(x, conv)
    return conv(x)


# ----------------------------------------------------------------------------- grouped convs
def grouped_dense_ok(x: torch.Tensor, conv: nn.Module) -> bool:
    """Training-time grouped (not depth-wise) convs, e.g. RegSeg's D-block 3 x 3s of group width 16
    (reference models/regseg.py:62-110).  MIOpen's grouped weight gradient in channels-last bf16
    is pathological at these shapes (tools/probe_grouped_conv.py), so such a conv runs as the
    dense conv of its block-diagonal weight: ``groups`` x the FLOPs of a conv that is tiny either
    way, on the routed kernels.  ``RTSEG_GROUPED_DENSE=0`` keeps MIOpen; so do
    ``RTSEG_DISABLE_HIP=1`` / ``RTSEG_HIP_OFF=conv`` (the stock yardstick runs the module's own
    grouped conv)."""
    return (isinstance(conv, nn.Conv2d) and 1 < conv.groups <= 32 and conv.groups != conv.in_channels
            and conv.padding_mode == "zeros" and not isinstance(conv.padding, str) and x.dim() == 4
            and x.is_cuda and torch.is_grad_enabled() and conv.weight.requires_grad
            and os.environ.get("RTSEG_GROUPED_DENSE", "1") != "0" and use_hip(x, "conv"))


_BLOCK_MASKS: dict = {}


def block_diagonal(w: torch.Tensor, groups: int) -> torch.Tensor:
    """[Cout, Cin/groups, KH, KW] grouped weight -> [Cout, Cin, KH, KW] dense (zeros off the
    diagonal blocks); its autograd backward sums the dense gradient's diagonal blocks back."""
    cout, cg = w.shape[0], w.shape[1]
    key = (cout, cg, groups, w.device, w.dtype)
    mask = _BLOCK_MASKS.get(key)
    if mask is None:
        og = cout // groups
        rows = torch.arange(cout, device=w.device)[:, None] // og
        cols = torch.arange(cg * groups, device=w.device)[None, :] // cg
        mask = _BLOCK_MASKS[key] = (rows == cols).to(w.dtype)[:, :, None, None]
    return w.repeat(1, groups, 1, 1) * mask


class _DenseView:
    """A conv seen as the dense conv of a derived ``weight`` -- a grouped conv's block-diagonal
    weight, or a zero-padded one (:func:`_apply`) -- for :class:`_ConvFn`, which reads geometry
    and the weight from the module it is given."""

    _rtseg_dense_view = True
    groups = 1
    bias = None
    padding_mode = "zeros"

    def __init__(self, conv: nn.Conv2d, weight: torch.Tensor):
        self.weight = weight
        self.stride, self.padding, self.dilation = conv.stride, conv.padding, conv.dilation
        self.kernel_size = conv.kernel_size
        self.out_channels, self.in_channels = weight.shape[0], weight.shape[1]
        self.training = conv.training


def padded_ok(conv: nn.Module) -> bool:
    """A spatial conv whose output channel count our kernels cannot store (Cout % 8 != 0, e.g.
    SegNet's 3 x 3 19-class classifier at full resolution, reference models/segnet.py) over a
    64-multiple input.  MIOpen's immediate-mode pick for its NHWC bf16 weight gradient ran for
    minutes (``profiles/r4_zoo/train_H_segnet_stall.txt``, ``tools/probe_conv_shapes.py``)."""
    return (conv.out_channels % 8 != 0 and conv.in_channels % 64 == 0 and max(conv.kernel_size) > 1
            and conv.groups == 1 and os.environ.get("RTSEG_PAD_COUT", "1") != "0")


def _apply(x: torch.Tensor, conv: nn.Module, stats: bool, store: bool = True):
    """:class:`_ConvFn` on ``conv``'s weight -> (y, statistics slab | None).  A :func:`padded_ok`
    conv runs on its weight zero-padded to the next 64 output channels (all three passes then
    fit the MFMA kernels) and returns the real channels as a dense channels-last tensor."""
    if not padded_ok(conv):
        return _ConvFn.apply(x, conv.weight, conv, stats, store)
    cp = -(-conv.out_channels // 64) * 64
    wp = F.pad(conv.weight, (0, 0, 0, 0, 0, 0, 0, cp - conv.out_channels))
    y, _ = _ConvFn.apply(x, wp, _DenseView(conv, wp), False, True)
    return y[:, :conv.out_channels].contiguous(memory_format=torch.channels_last), None


def grouped_as_dense(x: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
    from .bn import bias_add

    wd = block_diagonal(conv.weight, conv.groups)
    if (use_hip(x, "conv") and _mode() != "0" and _autocast_bf16(x) and x.stride(1) == 1
            and conv.kernel_size[0] * conv.kernel_size[1] <= 49):
        # channels-last, or a channel slice of it (RegSeg's split halves): one dense bf16 copy
        x = x.to(torch.bfloat16)
        if not x.is_contiguous(memory_format=torch.channels_last) or x.data_ptr() % 16:
            x = x.clone(memory_format=torch.channels_last)
        y, _ = _ConvFn.apply(x, wd, _DenseView(conv, wd), False, True)
        return bias_add(y, conv.bias) if conv.bias is not None else y
    return pruned_conv2d(x, wd, conv.bias, conv.stride, conv.padding, conv.dilation, 1)


def conv_bn_act(x: torch.Tensor, conv: nn.Module, bn: nn.Module, act="none", residual=None, act_module=None):
    """``act(bn(conv(x)) + residual)`` with the conv on our kernels where they win: BN statistics
    in its epilogue (training) or the whole BN + residual + activation tail (inference).  Any
    other case is ``conv`` followed by ``ops.bn_act``."""
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
                from .bn import bn_stats_begin

                y, part = conv_bn_stats(x, conv)
                # SyncBN: the statistics all-reduce leaves from the conv's epilogue slab right away
                # (async; None when not a multi-rank SyncBN) and bn_act waits at its finalize
                pending = bn_stats_begin(y, bn, part)
                return bn_act(y, bn, code, residual=residual, act_module=act_module, part=part, pending=pending)
    return bn_act(conv_forward(x, conv), bn, act, residual=residual, act_module=act_module)


class RoutedConv2d(PrunedConv2d):
    """A dense, bias-free ``nn.Conv2d`` that a model calls as a plain module (not through a
    ConvBNAct tail: e.g. ERFNet's last factorised conv, STDC's ``conv4`` / ``conv5``, decoder
    projections).  In bf16 training its three passes go through :class:`_ConvFn` -- each pass
    timed against MIOpen per shape like every other routed conv -- and in bf16 inference it
    reuses the cached bf16 weight (:func:`conv_forward`); anything else is the stock forward
    (dead taps dropped, :class:`PrunedConv2d`).  Same parameters and state-dict keys."""

    def forward(self, x):
        if (x.is_cuda and self.in_channels % 32 == 0 and (self.out_channels % 8 == 0 or padded_ok(self))
                and torch.is_grad_enabled()
                and self.weight.requires_grad and conv_ok(x, self)):
            x = x.to(torch.bfloat16)
            if x.data_ptr() % 16:  # the kernels' 16-byte operand loads
                x = x.clone(memory_format=torch.channels_last)
            return _apply(x, self, False)[0]
        if (x.is_cuda and not self.training and not torch.is_grad_enabled() and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            return conv_forward(x, self)  # its cached-weight branch (never falls through to self(x))
        return super().forward(x)


class GroupedConv2d(PrunedConv2d):
    """A grouped (not depth-wise) ``nn.Conv2d`` a model calls as a plain module -- ESPNetv2's EESP
    ``conv_init`` / ``conv_last`` (groups = 4, reference models/espnetv2.py): in bf16 training the
    block-diagonal dense route (:func:`grouped_as_dense`), otherwise the stock forward.  Same
    parameters and state-dict keys."""

    def forward(self, x):
        if grouped_dense_ok(x, self):
            return grouped_as_dense(x, self)
        return super().forward(x)


def routable(conv: nn.Module) -> bool:
    return (type(conv) in (nn.Conv2d, PrunedConv2d) and conv.groups == 1 and conv.bias is None
            and conv.padding_mode == "zeros" and not isinstance(conv.padding, str))


def convert_routed_convs(model: nn.Module) -> nn.Module:
    """Swap every remaining plain dense bias-free conv to :class:`RoutedConv2d` and every plain
    grouped one to :class:`GroupedConv2d` (in place, run after the other converters; parameters
    and checkpoint keys unchanged)."""
    for m in model.modules():
        if routable(m):
            m.__class__ = RoutedConv2d
        elif (type(m) in (nn.Conv2d, PrunedConv2d) and 1 < m.groups != m.in_channels
              and m.padding_mode == "zeros" and not isinstance(m.padding, str)):
            m.__class__ = GroupedConv2d
    return model


_ROUTED = (nn.Conv2d, PrunedConv2d, RoutedConv2d, GroupedConv2d)


def decisions() -> dict:
    """Per-shape kernel choices so far: key -> (index, name, [ms per candidate])."""
    return dict(_DECISIONS)
