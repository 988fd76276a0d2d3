"""GPU backend settings shared by every entry point (trainer, bench, FPS tool), so the training
run and the benchmark use the same MIOpen configuration.

* ``MIOPEN_USER_DB_PATH`` -> the in-tree ``miopen_db/`` (MIOpen's find results per conv shape on
  gfx950 travel with the repo; a fresh box reuses them instead of re-searching every solver);
* MIOpen's reference "naive" solvers are kept out of the exhaustive search (they take tens of
  seconds per shape at 1024x2048 and never win);
* ``torch.backends.cudnn.benchmark`` (MIOpen find mode) for the convs that stay on MIOpen
  (``config.cudnn_benchmark``, default on).

Environment variables already set by the user win.  Must run before the first convolution.
"""
from __future__ import annotations

import os

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_NAIVE = ("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD",
          "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW")


def configure_backend(benchmark: bool = True) -> None:
    for k in _NAIVE:
        os.environ.setdefault(k, "0")
    db = os.path.join(_REPO, "miopen_db")
    if os.path.isdir(db):
        os.environ.setdefault("MIOPEN_USER_DB_PATH", db)
    import torch

    torch.backends.cudnn.benchmark = bool(benchmark)
