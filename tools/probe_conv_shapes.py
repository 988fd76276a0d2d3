"""MIOpen time of every distinct conv shape of a zoo model, forward / data gradient / weight
gradient separately (bf16, channels-last, MIOpen immediate mode -- what a training run without
``--cudnn_benchmark`` gets).  Each line prints as soon as it is measured, so a shape on which
MIOpen falls back to a pathological kernel shows up as the last line of a run that stalls.

  python tools/probe_conv_shapes.py --model segnet --batch 8 --h 1024 --w 2048
"""
import argparse
import os
import sys
import time

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.models import get_model  # noqa: E402


def shapes_of(model, h, w, scale=8):
    """Conv shapes from a CPU forward at 1/scale resolution (the fused GPU tails call their conv
    kernels directly, past module hooks), scaled back up."""
    seen, hooks = {}, []
    for m in model.modules():
        if isinstance(m, nn.Conv2d):
            def hook(mod, inp, _out):
                x = inp[0]
                key = (mod.in_channels, mod.out_channels, mod.kernel_size, mod.stride, mod.padding, mod.dilation,
                       mod.groups, x.shape[2] * scale, x.shape[3] * scale)
                seen[key] = seen.get(key, 0) + 1
            hooks.append(m.register_forward_hook(hook))
    with torch.no_grad():
        model(torch.randn(1, 3, h // scale, w // scale))
    for hk in hooks:
        hk.remove()
    return seen


def timed(fn, reps=2):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="segnet")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--h", type=int, default=1024)
    ap.add_argument("--w", type=int, default=2048)
    a = ap.parse_args()
    c = BaseConfig()
    c.model, c.num_class = a.model, 19
    shapes = shapes_of(get_model(c).eval(), a.h, a.w)
    for key, count in sorted(shapes.items(), key=lambda kv: -kv[0][7] * kv[0][8]):
        cin, cout, k, s, p, d, g, h, w = key
        x = torch.randn(a.batch, cin, h, w, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        wt = torch.randn(cout, cin // g, *k, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.nn.functional.conv2d(x, wt, None, s, p, d, g)
        dy = torch.randn_like(y)

        def bwd(mask):
            return lambda: torch.ops.aten.convolution_backward(dy, x, wt, None, s, p, d, False, [0, 0], g, mask)

        print(f"{key} x{count}:", end="", flush=True)
        print(f" fwd {timed(lambda: torch.nn.functional.conv2d(x, wt, None, s, p, d, g)):.3f} ms", end="", flush=True)
        print(f" dgrad {timed(bwd([True, False, False])):.3f} ms", end="", flush=True)
        print(f" wgrad {timed(bwd([False, True, False])):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
