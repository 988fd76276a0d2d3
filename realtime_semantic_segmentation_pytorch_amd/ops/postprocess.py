"""Prediction post-processing on the HIP kernel of ``csrc/kernels/colorize.hip``.

Reference: core/seg_trainer.py:172-191 (argmax -> colormap -> optional PIL blend with the raw
image) and the argmax ONNX head of models/ddrnet.py:55-58.  :func:`colorize` returns the uint8
class map, the uint8 RGB colouring and (given the raw image) the blend, in one pass over the
logits; on CPU the same values come from the PyTorch formulation.
"""
from __future__ import annotations

import torch

from ._ext import ops, use_hip


def colorize_reference(logits, colormap, image=None, alpha=0.3):
    cls = logits.argmax(1)
    rgb = colormap[cls]
    blend = None
    if image is not None:
        a = image.float()  # fp32 multiply, add, truncate: PIL's Image.blend arithmetic
        blend = (a + (rgb.float() - a) * torch.tensor(alpha, dtype=torch.float32)).clamp(0, 255).to(torch.uint8)
    return cls.to(torch.uint8), rgb, blend


def colorize(logits: torch.Tensor, colormap: torch.Tensor, image: torch.Tensor | None = None,
             alpha: float = 0.3):
    """-> (class map uint8 [N,H,W], colours uint8 [N,H,W,3], blend uint8 [N,H,W,3] or None).

    ``colormap`` is uint8 ``[>= C, 3]``; ``image`` is the raw uint8 ``[N,H,W,3]`` image at the
    logits' resolution; the blend is ``image + alpha * (colour - image)``, bit-identical to PIL's.
    """
    if use_hip(logits) and logits.shape[1] <= 256:
        cls, rgb, blend = ops().colorize(logits, colormap.to(logits.device, torch.uint8).contiguous(),
                                         None if image is None else image.contiguous(), float(alpha))
        return cls, rgb, (blend if image is not None else None)
    return colorize_reference(logits, colormap, image, alpha)
