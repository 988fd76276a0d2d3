#!/usr/bin/env python3
"""Micro-benchmarks of the rtseg HIP ops vs their stock PyTorch/MIOpen equivalents.

Shapes are the DDRNet-23 layers at batch 8, 1024x2048 (the BASELINE config).
Reports time per call and effective HBM bandwidth (bytes the op must touch /
time).  Interleaves variants in one process (guide 5.4 rule 24).

  python tools/bench_ops.py [--only bn|interp|loss] [--reps 20]
"""
from __future__ import annotations

import argparse
import copy
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def bench_bn(reps):
    shapes = [(8, 64, 512, 1024), (8, 64, 256, 512), (8, 128, 128, 256), (8, 256, 64, 128),
              (8, 512, 32, 64), (8, 1024, 16, 32)]
    print(f"{'shape':>22} {'mode':>10} {'ours us':>9} {'torch us':>9} {'ours GB/s':>10} {'speedup':>8}")
    for shp in shapes:
        x = torch.randn(shp, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        res = torch.randn_like(x)
        bn = nn.BatchNorm2d(shp[1]).cuda()
        bn_t = copy.deepcopy(bn)
        nbytes = x.numel() * 2
        for mode in ("relu", "res+relu"):
            r = res if mode == "res+relu" else None
            xg = x.detach().requires_grad_(True)
            rg = r.detach().requires_grad_(True) if r is not None else None

            def ours_f():
                return ops.bn_act(xg, bn, "relu", residual=rg)

            def torch_f():
                y = bn_t(xg)
                if rg is not None:
                    y = y + rg
                return torch.relu(y)
            tf_o = timeit(ours_f, reps)
            tf_t = timeit(torch_f, reps)
            # forward bytes: read x twice (stats + apply) (+res) + write y
            fb = nbytes * (3 + (1 if r is not None else 0))
            print(f"{str(shp):>22} {'fwd ' + mode:>10} {tf_o:9.1f} {tf_t:9.1f} {fb / tf_o / 1e3:10.0f} {tf_t / tf_o:8.2f}")
            yo, yt = ours_f(), torch_f()
            g = torch.randn_like(yo)

            def ours_b():
                torch.autograd.grad(yo, [xg] + ([rg] if rg is not None else []), g, retain_graph=True)

            def torch_b():
                torch.autograd.grad(yt, [xg] + ([rg] if rg is not None else []), g, retain_graph=True)
            tb_o = timeit(ours_b, reps)
            tb_t = timeit(torch_b, reps)
            bb = nbytes * (5 + (3 if r is not None else 0))
            print(f"{str(shp):>22} {'bwd ' + mode:>10} {tb_o:9.1f} {tb_t:9.1f} {bb / tb_o / 1e3:10.0f} {tb_t / tb_o:8.2f}")


def bench_interp(reps):
    import torch.nn.functional as F
    cases = [((8, 128, 64, 128), (128, 256)), ((8, 256, 16, 32), (128, 256)), ((8, 19, 128, 256), (1024, 2048))]
    for shp, size in cases:
        x = torch.randn(shp, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        skip = torch.randn(shp[0], shp[1], *size, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        o = timeit(lambda: ops.interpolate(x, size, True, skip=skip, act="relu"), reps)
        t = timeit(lambda: torch.relu(F.interpolate(x, size, mode="bilinear", align_corners=True) + skip), reps)
        by = (x.numel() + 2 * skip.numel()) * 2
        print(f"interp fwd {str(shp):>20}->{size}: ours {o:8.1f} us ({by / o / 1e3:.0f} GB/s)  torch {t:8.1f} us")
        xg = x.detach().requires_grad_(True)
        yo = ops.interpolate(xg, size, True)
        yt = F.interpolate(xg, size, mode="bilinear", align_corners=True)
        g = torch.randn_like(yo)
        o = timeit(lambda: torch.autograd.grad(yo, xg, g, retain_graph=True), reps)
        t = timeit(lambda: torch.autograd.grad(yt, xg, g, retain_graph=True), reps)
        print(f"interp bwd {str(shp):>20}->{size}: ours {o:8.1f} us  torch {t:8.1f} us")


def bench_loss(reps):
    import torch.nn.functional as F
    logits = torch.randn(8, 19, 128, 256, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    labels = torch.randint(0, 19, (8, 1024, 2048), device="cuda")
    o = timeit(lambda: ops.seg_cross_entropy(logits, labels), reps)
    lo = ops.seg_cross_entropy(logits, labels)
    ob = timeit(lambda: torch.autograd.grad(lo, logits, retain_graph=True), reps)

    def ref():
        up = F.interpolate(logits, (1024, 2048), mode="bilinear", align_corners=True)
        return F.cross_entropy(up.float(), labels, ignore_index=255)
    t = timeit(ref, reps)
    lt = ref()
    tb = timeit(lambda: torch.autograd.grad(lt, logits, retain_graph=True), reps)
    print(f"fused upsample+OHEM-CE fwd {o:8.1f} us bwd {ob:8.1f} us | torch upsample+CE fwd {t:8.1f} us bwd {tb:8.1f} us")
    aux = torch.randn(8, 19, 128, 256, device="cuda", dtype=torch.bfloat16).requires_grad_(True)
    o = timeit(lambda: ops.seg_cross_entropy(aux, labels, resize_logits=False), reps)
    print(f"aux (nearest labels) fwd {o:8.1f} us")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="all")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    assert ops.load()
    if a.only in ("all", "bn"):
        bench_bn(a.reps)
    if a.only in ("all", "interp"):
        bench_interp(a.reps)
    if a.only in ("all", "loss"):
        bench_loss(a.reps)


if __name__ == "__main__":
    main()
