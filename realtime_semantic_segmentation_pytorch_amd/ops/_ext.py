"""Loader for the in-tree HIP extension (``_C/librtseg_hip.so``).

Policy (see README "Kernel dispatch"):
* GPU tensors ALWAYS run the HIP kernels.  If the library cannot be loaded on a
  machine that has a GPU, ops raise instead of silently falling back.
* CPU tensors run the PyTorch reference formulation of the same op (used by the
  CPU test-suite and the CPU plumbing config, and as the numerics oracle).
* ``RTSEG_DISABLE_HIP=1`` is an explicit opt-out used only for A/B benchmarks.
"""
from __future__ import annotations

import os
import threading

import torch

from . import build as _build

_lock = threading.Lock()
_loaded = False
_load_error: Exception | None = None


def hip_disabled() -> bool:
    return os.environ.get("RTSEG_DISABLE_HIP", "0") == "1"


def load(build_if_missing: bool = True) -> bool:
    """Load (building first if needed) the extension. Returns True on success."""
    global _loaded, _load_error
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        try:
            path = _build.LIB_PATH
            override = os.environ.get("RTSEG_LIB_PATH")  # a prebuilt library (A/B of two builds)
            if override:
                path, build_if_missing = override, False
            if build_if_missing:
                try:
                    path = _build.build()
                except Exception as e:  # build tools absent: use a prebuilt library if present
                    if not os.path.exists(path):
                        raise e
            torch.ops.load_library(path)
            _loaded = True
            _load_error = None
        except Exception as e:  # pragma: no cover - exercised on broken installs
            _load_error = e
    return _loaded


# Raw-pointer writers (the fused optimizer step, the EMA lerp) update parameters, EMA weights
# and BN running statistics without bumping their autograd ``_version`` counters.  Every cache
# keyed on (data_ptr, _version) -- the bf16 weight copies of ops.conv, BN eval coefficients of
# ops.bn -- also folds in this generation, which those writers advance after each launch.
_WRITE_GEN = [0]


def bump_write_generation() -> None:
    _WRITE_GEN[0] += 1


def write_generation() -> int:
    return _WRITE_GEN[0]


def library_path() -> str:
    return _build.LIB_PATH


def families_off() -> frozenset:
    """``RTSEG_HIP_OFF=bn,interp,...``: kernel families sent to their stock PyTorch formulation
    (numerics bisection, tools/probe_numerics_bisect.py).  Families: act, bn, conv, deconv, detail,
    dilated, dw, gate, interp, kd, loss, pool, shuffle, tapconv."""
    raw = os.environ.get("RTSEG_HIP_OFF", "")
    return frozenset(f.strip() for f in raw.split(",") if f.strip())


def use_hip(t: torch.Tensor, family: str | None = None) -> bool:
    """Whether an op on tensor ``t`` must take the HIP path (raises if unavailable)."""
    if not t.is_cuda or hip_disabled():
        return False
    if family is not None and family in families_off():
        return False
    if not load():
        raise RuntimeError(
            "rtseg HIP extension is required for GPU tensors but failed to load: "
            f"{_load_error!r}. Build it with `python -m realtime_semantic_segmentation_pytorch_amd.ops.build`.")
    return True


class _TracedOps:
    """``RTSEG_TRACE_OPS=<file>``: every rtseg op call is logged (name, tensor shapes/dtypes,
    data pointers) to ``<file>`` BEFORE it launches and the device is synchronised after it,
    so the last line written before a GPU fault names the faulting op (used with the
    guard-page allocator, ``utils/guard.py``)."""

    def __init__(self, path):
        self._f = open(path, "a", buffering=1)
        self._n = 0

    def __getattr__(self, name):
        fn = getattr(torch.ops.rtseg, name)

        def call(*args, **kw):
            self._n += 1
            desc = []
            for a in list(args) + list(kw.values()):
                if isinstance(a, torch.Tensor):
                    desc.append(f"T{tuple(a.shape)}{str(a.dtype)[6:]}@{a.data_ptr():x}"
                                f"{'' if a.is_contiguous() else '/cl' if a.dim() == 4 and a.is_contiguous(memory_format=torch.channels_last) else '/nc'}")
                elif isinstance(a, (int, float, bool)) or a is None:
                    desc.append(repr(a))
                else:
                    desc.append(type(a).__name__)
            self._f.write(f"{self._n} {name}({', '.join(desc)})\n")
            os.fsync(self._f.fileno())
            out = fn(*args, **kw)
            # a synchronize is illegal while a HIP graph is being captured (graph_step, the
            # inference engines): there the trace line is still written, the sync skipped
            if not torch.cuda.is_current_stream_capturing():
                torch.cuda.synchronize()
            return out

        return call


_traced = None


def ops():
    global _traced
    path = os.environ.get("RTSEG_TRACE_OPS")
    if path:
        if _traced is None:
            _traced = _TracedOps(path)
        return _traced
    return torch.ops.rtseg
