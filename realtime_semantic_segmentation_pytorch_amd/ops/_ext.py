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


def library_path() -> str:
    return _build.LIB_PATH


def use_hip(t: torch.Tensor) -> bool:
    """Whether an op on tensor ``t`` must take the HIP path (raises if unavailable)."""
    if not t.is_cuda or hip_disabled():
        return False
    if not load():
        raise RuntimeError(
            "rtseg HIP extension is required for GPU tensors but failed to load: "
            f"{_load_error!r}. Build it with `python -m realtime_semantic_segmentation_pytorch_amd.ops.build`.")
    return True


def ops():
    return torch.ops.rtseg
