#!/usr/bin/env python3
"""Effective HBM bandwidth of each BatchNorm pass on the DDRNet-23 batch-32 layer shapes.

Every pass is timed alone (CUDA events, interleaved repetitions) and reported as bytes the pass
must touch / time, next to a plain device copy of the same tensor (the practical streaming
ceiling).  Passes: ``apply`` (relu, no residual), ``apply_bits`` (residual + relu + derivative
bit mask), ``bwd_reduce`` (slab of sum g, sum g(x-mean); mask from x), ``bwd_full`` (reduce +
apply: dx), ``bwd_full_bits`` (bit mask + residual gradient).

  python tools/bench_bn_bw.py [--reps 10] [--batch 32]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / reps)
    return best * 1e3  # us


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--batch", type=int, default=32)
    a = p.parse_args()
    assert ops.load(), "rtseg extension missing"
    o = torch.ops.rtseg
    n = a.batch
    shapes = [(n, 64, 512, 1024), (n, 64, 256, 512), (n, 128, 128, 256), (n, 256, 64, 128), (n, 512, 32, 64),
              (8, 19, 1024, 2048)]  # the full-resolution 19-class head of the DeConvBNAct models (batch 8)
    print(f"{'shape':>24} {'pass':>14} {'us':>9} {'GB/s':>7} {'copy GB/s':>9}")
    for shp in shapes:
        C = shp[1]
        x = torch.randn(shp, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        res = torch.randn_like(x)
        dy = torch.randn_like(x)
        w = torch.rand(C, device="cuda") + 0.5
        b = torch.randn(C, device="cuda") * 0.1
        mi, ss, fs = o.bn_stats_finalize(x, w, b, None, None, None, 0.1, 1e-5)
        _, bits = o.bn_apply_bits(x, ss, res, 1)
        nb = x.numel() * 2
        tc = timeit(lambda: x.clone(memory_format=torch.channels_last), a.reps)
        copy_bw = 2 * nb / tc / 1e3
        rows = [
            ("apply", lambda: o.bn_apply(x, ss, None, 1), 2 * nb),
            ("apply_bits", lambda: o.bn_apply_bits(x, ss, res, 1), 3 * nb + nb // 16),
            ("bwd_reduce", lambda: o.bn_bwd_sums(dy, x, None, mi, ss, 1, 2), 2 * nb),
            ("bwd_full", lambda: o.bn_backward(dy, x, None, None, fs, mi, ss, w, 1, 2, False, True, True, None),
             5 * nb),
            ("bwd_full_bits", lambda: o.bn_backward(dy, x, bits, None, fs, mi, ss, w, 1, 3, True, True, True,
                                                    None), 6 * nb + 2 * (nb // 16)),
        ]
        for name, fn, nbytes in rows:
            t = timeit(fn, a.reps)
            print(f"{str(shp):>24} {name:>14} {t:9.1f} {nbytes / t / 1e3:7.0f} {copy_bw:9.0f}", flush=True)
        del x, res, dy, bits
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
