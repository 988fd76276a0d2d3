#!/usr/bin/env python3
"""Can a conv weight gradient overlap the BatchNorm backward on a second HIP stream?

DDRNet-23 layer shapes at batch 32.  Times (CUDA events, best of 3 x reps):
* A: ``conv_whalo_wgrad`` (3x3, MFMA-bound-ish) alone;
* B: the fused BN backward (reduce + apply, relu, mask from x; memory-bound) alone;
* A on stream 1 and B on stream 2, issued back to back, together.
``overlap`` = (A + B - together) / min(A, B): 1 = the shorter one hidden entirely.

  python tools/probe_overlap.py [--reps 10]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402


def best(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = float("inf")
    for _ in range(3):
        torch.cuda.synchronize()
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        out = min(out, s.elapsed_time(e) / reps)
    return out * 1e3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=10)
    a = p.parse_args()
    assert ops.load()
    o = torch.ops.rtseg
    cl = torch.channels_last
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    print(f"{'layer':>22} {'A wgrad us':>11} {'B bnbwd us':>11} {'A||B us':>9} {'overlap':>8}")
    for n, c, h, w in [(32, 64, 256, 512), (32, 128, 128, 256), (32, 256, 64, 128)]:
        x = torch.randn(n, c, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        dy = torch.randn_like(x)
        bn = ops.convert_batchnorm(nn.Sequential(nn.BatchNorm2d(c))).cuda()[0].train()
        xr = x.clone().requires_grad_(True)
        y = ops.bn_act(xr, bn, "relu")

        def A():
            o.conv_whalo_wgrad(x, dy, 3, 3, [1, 1], [1, 1], [1, 1], True)

        def B():
            torch.autograd.grad(y, xr, dy, retain_graph=True)

        def AB():
            cur = torch.cuda.current_stream()
            s1.wait_stream(cur)
            s2.wait_stream(cur)
            with torch.cuda.stream(s1):
                A()
            with torch.cuda.stream(s2):
                B()
            cur.wait_stream(s1)
            cur.wait_stream(s2)

        ta, tb, tab = best(A, a.reps), best(B, a.reps), best(AB, a.reps)
        ov = (ta + tb - tab) / min(ta, tb)
        print(f"{str((n, c, h, w)):>22} {ta:11.1f} {tb:11.1f} {tab:9.1f} {ov:8.2f}", flush=True)


if __name__ == "__main__":
    main()
