"""Parameter and MAC counting (reference tools/get_model_infos.py uses ptflops, absent here).

MACs are counted with forward hooks on convolution / transposed convolution
/ linear modules (the layers ptflops counts; like ptflops, functional ops
such as ``F.interpolate`` are not counted).
"""
from __future__ import annotations

import torch
import torch.nn as nn


def count_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())


@torch.no_grad()
def count_macs(model: nn.Module, input_shape=(1, 3, 512, 1024)) -> int:
    total = [0]

    def conv_hook(m, inp, out):
        k = m.weight.shape[2] * m.weight.shape[3]
        cin_per_group = m.in_channels // m.groups
        if isinstance(m, nn.ConvTranspose2d):
            total[0] += inp[0].numel() * k * (m.out_channels // m.groups)
        else:
            total[0] += out.numel() * k * cin_per_group
        if m.bias is not None:
            total[0] += out.numel()

    def linear_hook(m, inp, out):
        total[0] += out.numel() * m.in_features

    hooks = []
    for m in model.modules():
        if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
            hooks.append(m.register_forward_hook(conv_hook))
        elif isinstance(m, nn.Linear):
            hooks.append(m.register_forward_hook(linear_hook))
    was_training = model.training
    model.eval()
    p = next(model.parameters())
    try:
        model(torch.zeros(*input_shape, device=p.device, dtype=p.dtype))
    finally:
        for h in hooks:
            h.remove()
        model.train(was_training)
    return total[0]
