#!/usr/bin/env python3
"""A/B of the fused upsample + OHEM cross-entropy backward forms on the headline shape: DDRNet-23's
main head, batch 32, logits [32, 19, 128, 256] bf16 channels-last, uint8 labels 1024 x 2048.
RTSEG_LOSS_BWD_RUN selects the form per launch (0 round-4 tile, 1 first run form, 2 packed run
form); forms are interleaved in one process and the gradients compared with each other.

  python tools/bench_loss_bwd.py [--reps 20] [--batch 32]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--forms", default="1,2")
    a = ap.parse_args()
    assert ops.load()
    torch.manual_seed(0)
    logits = torch.randn(a.batch, 19, 128, 256, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    labels = torch.randint(0, 19, (a.batch, 1024, 2048), device="cuda", dtype=torch.uint8)
    labels[torch.rand(labels.shape, device="cuda") < 0.1] = 255
    loss = ops.seg_cross_entropy(logits, labels)
    forms = a.forms.split(",")
    grads, times = {}, {f: [] for f in forms}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(3):
        for f in forms:
            os.environ["RTSEG_LOSS_BWD_RUN"] = f
            for _ in range(3):
                torch.autograd.grad(loss, logits, retain_graph=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(a.reps):
                g, = torch.autograd.grad(loss, logits, retain_graph=True)
            e.record()
            torch.cuda.synchronize()
            times[f].append(s.elapsed_time(e) / a.reps * 1e3)
            grads[f] = g.float()
    for f in forms:
        print(f"form {f}: backward {min(times[f]):8.1f} us (rounds {', '.join(f'{t:.1f}' for t in times[f])})")
    base = grads[forms[0]]
    for f in forms[1:]:
        d = (grads[f] - base).abs().max().item()
        print(f"max |grad[{f}] - grad[{forms[0]}]| = {d:.3e} (max |grad| {base.abs().max().item():.3e})")


if __name__ == "__main__":
    main()
