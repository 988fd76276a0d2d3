"""Guard-page allocator switch (debugging; ``csrc/tools/guard_alloc.cpp``).

``install("tail")`` makes every device tensor END at an unmapped guard page, ``install("head")``
makes it START right after one, so an out-of-bounds access of any kernel faults on the first
launch that does it instead of depending on what the caching allocator placed next to the
tensor.  Must run before the process allocates its first CUDA tensor.  Combine with
``RTSEG_TRACE_OPS=<file>`` (``ops/_ext.py``) to name the op that faulted.

Limitation (measured on MI355X, profiles/r3_fault/README.md): the vendor libraries do not work
on memory of the HIP virtual-memory API -- a hipBLASLt/rocBLAS ``mm`` returns wrong results
(tools/guard_sanity.py: relative error 0.30) and MIOpen convolutions garbage -- so the guard
is only meaningful for workloads made of our kernels and elementwise ATen ops.  It is NOT part
of the test suite (a wrong GEMM upstream can turn into an index kernel's fault downstream)."""
from __future__ import annotations

import ctypes
import os

import torch

_installed = None


def install(mode: str = "tail") -> str:
    global _installed
    if _installed is not None:
        if _installed != mode:
            raise RuntimeError(f"guard allocator already installed in {_installed!r} mode")
        return mode
    if mode not in ("tail", "head"):
        raise ValueError(mode)
    from ..ops import build

    path = build.build_guard()
    os.environ["RTSEG_GUARD_MODE"] = mode
    alloc = torch.cuda.memory.CUDAPluggableAllocator(path, "rtseg_guard_malloc", "rtseg_guard_free")
    torch.cuda.memory.change_current_allocator(alloc)
    # MIOpen's convolutions return garbage on memory of the HIP virtual-memory API (measured:
    # tools/probe_guard_diff.py); PyTorch's own convolutions are correct there (GEMMs are not)
    torch.backends.cudnn.enabled = False
    _installed = mode
    return mode


def stats() -> dict:
    """Allocations made, live / peak mapped bytes and the mapping granularity."""
    from ..ops import build

    lib = ctypes.CDLL(build.GUARD_LIB_PATH)
    out = (ctypes.c_size_t * 4)()
    lib.rtseg_guard_stats(out)
    return {"allocs": out[0], "live_bytes": out[1], "peak_bytes": out[2], "granularity": out[3]}
