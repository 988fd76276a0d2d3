"""Which aten ops of a training step move large tensors outside the HIP kernels?  Used by bench.py
with RTSEG_PROBE_OPS=<out file>: one extra step runs under a TorchDispatchMode (forward and
backward) that records every copy / cast / fill / add / mul-style op over more than ``min_numel``
elements, by (op, shapes, dtypes, innermost package source line), with the call count.
"""
from __future__ import annotations

import collections
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

PKG = "realtime_semantic_segmentation_pytorch_amd"
WATCH = ("copy", "_to_copy", "clone", "contiguous", "fill", "zero", "add", "mul", "sub", "cat", "where",
         "masked", "index", "sum", "mean", "div", "neg", "relu", "threshold", "empty_like", "zeros", "ones")


def _site():
    for fr in reversed(traceback.extract_stack()[:-3]):
        if PKG in fr.filename and "/ops/" not in fr.filename:
            return f"{fr.filename.split(PKG + '/')[-1]}:{fr.lineno}"
    for fr in reversed(traceback.extract_stack()[:-3]):
        if PKG in fr.filename:
            return f"{fr.filename.split(PKG + '/')[-1]}:{fr.lineno}"
    return "?"


class OpProbe(TorchDispatchMode):
    def __init__(self, min_numel=1 << 20):
        super().__init__()
        self.min_numel = min_numel
        self.hits = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func.overloadpacket.__name__)
        if any(w in name for w in WATCH):
            ts = [a for a in args if isinstance(a, torch.Tensor)]
            outs = out if isinstance(out, (tuple, list)) else [out]
            outs = [o for o in outs if isinstance(o, torch.Tensor)]
            big = max([t.numel() for t in ts + outs] + [0])
            if big >= self.min_numel:
                shapes = tuple(tuple(t.shape) for t in ts[:2])
                dts = tuple(str(t.dtype)[6:] for t in ts[:2] + outs[:1])
                site = _site()
                if site == "?":  # backward engine: name the autograd node that produced the operand
                    node = torch._C._current_autograd_node()
                    if node is not None:
                        nxt = [type(f).__name__ if f is not None else "-" for f, _ in node.next_functions][:3]
                        site = f"bwd:{node.name()}->{','.join(nxt)}"
                self.hits[(name, shapes, dts, site)] += 1
        return out

    def report(self) -> str:
        lines = []
        for (name, shapes, dts, site), n in self.hits.most_common(80):
            lines.append(f"{n:4d}  {name:28s} {str(shapes):60s} {str(dts):34s} {site}")
        return "\n".join(lines) + "\n"
