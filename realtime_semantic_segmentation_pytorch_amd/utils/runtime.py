"""GPU backend settings shared by every entry point (trainer, bench, FPS tool), so the training
run and the benchmark use the same MIOpen configuration.

* ``MIOPEN_USER_DB_PATH`` -> the in-tree ``miopen_db/`` (MIOpen's find results per conv shape on
  gfx950 travel with the repo; a fresh box reuses them instead of re-searching every solver);
* MIOpen's reference "naive" solvers are kept out of the exhaustive search only by bench.py
  (they take tens of seconds per shape at 1024x2048 and never win there, but they are the
  fallback for the zoo's degenerate dilated convs, so a trainer process keeps them);
* ``torch.backends.cudnn.benchmark`` (MIOpen find mode) for the convs that stay on MIOpen
  (``config.cudnn_benchmark``) on the models it is verified for.  OFF by default since round 4:
  a BiSeNetV2 training run at a new shape (batch 8, 256 x 512) left the GPU faulted in its first
  backward, where find mode runs MIOpen's exhaustive solver search on every new shape (the
  fault class of rounds 1-3, profiles/r3_fault).  bench.py turns it on for its one config,
  whose shapes have run the search without a fault in every round; elsewhere MIOpen runs in
  immediate mode (the find database in ``miopen_db/`` where it has the shape, else heuristics).

* ``config.deterministic``: bit-reproducible training steps, run to run and process to process
  (``RTSEG_DETERMINISTIC=1``): conv kernels from the tuning database or a fixed rule, never a
  timing (ops/conv.py ``_choose``), and MIOpen's deterministic solvers only.  The HIP kernels
  are deterministic without it: BN / wgrad / loss partial sums are per-block slabs reduced in a
  fixed order, and the loss backward's border atomics are split into launches in which no cell
  has two writers (seg_loss.hip).

Environment variables already set by the user win.  Must run before the first convolution.
"""
from __future__ import annotations

import os

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_NAIVE = ("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD",
          "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW")


# Models whose MIOpen find (exhaustive solver search) has been verified on gfx950 at training and
# inference shapes.  Elsewhere find mode stays off: the zoo has degenerate dilated geometries
# (LEDNet's (3, 1) convs with dilation 17 on a 16-row map at 128 x 256, CFPNet's dilation-16
# convs) on which some NHWC solvers fault the GPU during the search (profiles/r1_zoo_fps,
# tools/test_speed.py), and the find choice would persist for the whole process.
FIND_VERIFIED = ("ddrnet", "bisenetv2", "stdc", "pp_liteseg", "ppliteseg")


def configure_backend(benchmark: bool = True, model=None, exclude_naive: bool = False,
                      deterministic: bool = False) -> None:
    """MIOpen setup.  ``benchmark``: find mode, honoured only for ``FIND_VERIFIED`` models (and
    always reset otherwise, so a process that trains several models never carries find mode
    over to an unverified one).  ``exclude_naive``: keep MIOpen's naive solvers out of the
    search -- only for single-model processes on verified shapes (bench.py): the setting is
    read once per process and the naive solvers are the fallback for degenerate geometries."""
    if exclude_naive:
        for k in _NAIVE:
            os.environ.setdefault(k, "0")
    db = os.path.join(_REPO, "miopen_db")
    if os.path.isdir(db):
        os.environ.setdefault("MIOPEN_USER_DB_PATH", db)
    import torch

    verified = model is None or str(model).lower() in FIND_VERIFIED
    torch.backends.cudnn.benchmark = bool(benchmark) and verified and not deterministic
    if deterministic:
        os.environ["RTSEG_DETERMINISTIC"] = "1"
        torch.backends.cudnn.deterministic = True
