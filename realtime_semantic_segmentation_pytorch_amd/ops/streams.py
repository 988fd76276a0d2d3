"""Concurrent model branches on a second HIP stream (inference).

At batch 1 most layers of a two-branch network launch grids that do not fill 256 CUs: DDRNet-23's
high-resolution branch (1/8, 128 channels) and low-resolution branch (1/16 - 1/32, 256 - 512
channels) each run tens of 10 - 50 us kernels back to back (profiles/r6_infer).  The branches
are independent between fusions (reference models/ddrnet.py:41-47, 57-63), so
:func:`concurrent_branches` runs one of them on a side stream: the two kernel streams share the
CUs.  Inside a HIP-graph capture (utils/inference.py) the fork / join become graph edges, so the
replayed graph keeps the concurrency at no host cost.

Only without autograd (inference / validation): in training the branches stay on one stream,
where the batch already fills the GPU and autograd's stream semantics would need every saved
tensor re-recorded.

Measured (profiles/r6_infer, DDRNet-23 bf16 batch 1, 1024 x 2048): +8.7 % (722 -> 786 FPS) while
the low-resolution layers ran on 256-pixel tiles; after the small-tile / split-K inference
kernels (ops/conv.py conv_bn_act_eval) fill the CUs on their own it is neutral (905 / 908 on,
906 / 909 off).  So it is opt-in: ``RTSEG_BRANCH_STREAMS=1``.
"""
from __future__ import annotations

import os
from typing import Any, Callable, Dict, Tuple

import torch

_ON = os.environ.get("RTSEG_BRANCH_STREAMS", "0") == "1"
_SIDE: Dict[int, torch.cuda.Stream] = {}
FORKS = [0]  # concurrent launches issued (tests)


def _side(device: torch.device) -> torch.cuda.Stream:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _SIDE.get(idx)
    if s is None:
        s = _SIDE[idx] = torch.cuda.Stream(device=idx)
    return s


def concurrent_branches(fa: Callable[[], Any], fb: Callable[[], Any], device: torch.device) -> Tuple[Any, Any]:
    """``(fa(), fb())`` with ``fb`` on a side stream when no autograd graph is recorded.  The
    caller keeps ``fb``'s inputs alive until this returns (they are read on the side stream);
    ``fb``'s output (a tensor or a list / tuple of tensors) is recorded on the current stream,
    which waits for the side stream."""
    if not _ON or torch.is_grad_enabled() or device.type != "cuda":
        return fa(), fb()
    main = torch.cuda.current_stream(device)
    side = _side(device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        b = fb()
    a = fa()
    main.wait_stream(side)
    for t in (b if isinstance(b, (list, tuple)) else (b,)):
        t.record_stream(main)
    FORKS[0] += 1
    return a, b
