"""Graph-captured inference engine (the MI355X-native replacement for the
reference's eager ``model(input)`` loop in tools/test_speed.py:26-60).

A segmentation forward at batch 1 is a few hundred small kernels; launched
eagerly from Python the host becomes the bottleneck.  ``InferenceEngine``
puts the model in eval / channels-last / (bf16) form, warms it up on a side
stream (MIOpen solver selection happens here), then captures ONE forward into
a HIP graph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) with static
input/output buffers.  ``engine(x)`` is a device copy into the static input +
one graph launch.  All rtseg HIP ops are capture-safe (no host syncs, stream-
ordered, caching-allocator memory).
"""
from __future__ import annotations

import copy
from typing import Optional, Sequence

import torch
import torch.nn as nn

from ..ops.act import _HipAct

from .. import ops


class InferenceEngine:
    def __init__(self, model: nn.Module, input_shape: Sequence[int], dtype: torch.dtype = torch.bfloat16,
                 channels_last: bool = True, use_graph: bool = True, warmup: int = 3,
                 device: Optional[torch.device] = None, cast_weights: bool = True,
                 input_dtype: Optional[torch.dtype] = None):
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.dtype = dtype
        self.channels_last = channels_last
        self.autocast = dtype in (torch.bfloat16, torch.float16)
        if self.autocast and cast_weights:
            # autocast re-casts every fp32 conv / linear (and PReLU) weight on every forward (one extra
            # kernel per layer inside the graph: 18 % of CGNet's bf16 replay time); cast them
            # once, on a private copy so the caller's fp32 model is untouched
            model = copy.deepcopy(model)
            for m in model.modules():
                # isinstance: the rtseg conv subclasses (DilatedGroupConv2d, DepthwiseConv2d, ...)
                # carry fp32 weights too
                # (the HIP activation kernels read an fp32 PReLU weight directly: no autocast cast)
                if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d, nn.Linear)) or (
                        isinstance(m, nn.PReLU) and not isinstance(m, _HipAct)):
                    m.to(dtype)
        self.model = model.eval().to(self.device)
        if channels_last:
            self.model = self.model.to(memory_format=torch.channels_last)
        fmt = torch.channels_last if channels_last else torch.contiguous_format
        # by default a reduced-precision engine takes its input in that dtype: the copy into the
        # static buffer casts, and image-side ops (input pyramids, pooled image shortcuts, resized
        # inputs) run in bf16 instead of leaving fp32 islands that every consumer conv casts again.
        # The image is then rounded once before the model (the first conv rounds it under
        # autocast anyway); tests/test_misc_ops_gpu.py bounds the effect on the models with image-
        # side ops (DFANet, ESPNet, ICNet).  ``input_dtype=torch.float32`` keeps the eager path's
        # fp32 image exactly.
        in_dt = input_dtype or (dtype if self.autocast else torch.float32)
        self.static_in = torch.zeros(*input_shape, device=self.device, dtype=in_dt).contiguous(memory_format=fmt)
        self.graph = None
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(max(1, warmup)):
                out = self._forward(self.static_in)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self.static_out = out
        if use_graph:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.static_out = self._forward(self.static_in)
            torch.cuda.synchronize(self.device)

    @torch.no_grad()
    def _forward(self, x):
        with torch.autocast("cuda", dtype=self.dtype, enabled=self.autocast):
            out = self.model(x)
        if isinstance(out, (tuple, list)):
            out = out[0]
        return ops.materialize(out)

    @torch.no_grad()
    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if self.graph is None:
            return self._forward(x.to(self.device, non_blocking=True).contiguous(
                memory_format=torch.channels_last if self.channels_last else torch.contiguous_format))
        self.static_in.copy_(x, non_blocking=True)
        self.graph.replay()
        return self.static_out

    @torch.no_grad()
    def predict(self, x: torch.Tensor) -> torch.Tensor:
        """Class-index map [N, H, W] (argmax over classes)."""
        return self(x).argmax(dim=1)
