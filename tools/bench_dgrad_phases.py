#!/usr/bin/env python3
"""A/B of the igemm data gradient of strided convs: one launch per output phase vs every phase in
one launch (fused_phases=True), on DDRNet-23's b32 strided shapes, with and without an addend.

  python tools/bench_dgrad_phases.py [--batch 32]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402

# (cin, h, w, cout, k, stride): forward geometry
SHAPES = [(64, 512, 1024, 64, 3, 2), (64, 256, 512, 128, 3, 2), (128, 128, 256, 256, 3, 2),
          (256, 64, 128, 512, 3, 2), (512, 32, 64, 512, 3, 2), (128, 128, 256, 512, 3, 4),
          (64, 256, 512, 128, 1, 2), (512, 32, 64, 1024, 1, 2)]


def timeit(fn, reps=10):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    assert ops.load()
    r = torch.ops.rtseg
    cl = dict(memory_format=torch.channels_last)
    for cin, h, w, cout, k, s in SHAPES:
        p = (k - 1) // 2
        ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        wt = (torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).to(torch.bfloat16)
        wtr = wt.permute(1, 2, 3, 0).contiguous()
        dy = torch.randn(a.batch, cout, ho, wo, device="cuda", dtype=torch.bfloat16).contiguous(**cl)
        add = torch.randn(a.batch, cin, h, w, device="cuda", dtype=torch.bfloat16).contiguous(**cl)
        xs = [a.batch, cin, h, w]
        for addend in (None, add):
            best = {}
            for rnd in range(3):
                for fused in (False, True):
                    fn = lambda: r.conv_igemm_dgrad(dy, wtr, xs, [s, s], [p, p], [1, 1], None, addend, None, None, fused)
                    if rnd == 0:
                        fn()
                    best[fused] = min(best.get(fused, float("inf")), timeit(fn))
            same = torch.equal(r.conv_igemm_dgrad(dy, wtr, xs, [s, s], [p, p], [1, 1], None, addend, None, None, True),
                               r.conv_igemm_dgrad(dy, wtr, xs, [s, s], [p, p], [1, 1], None, addend, None, None, False))
            tag = "+addend" if addend is not None else ""
            print(f"{cin}->{cout} k{k} s{s} @ {h}x{w}{tag:8s} phases {best[False]:8.1f} us  fused {best[True]:8.1f} us "
                  f"({best[False] / best[True]:.2f}x)  equal={same}", flush=True)
        del add, dy


if __name__ == "__main__":
    main()
