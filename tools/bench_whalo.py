#!/usr/bin/env python3
"""conv_whalo weight gradient, variant 1 vs 2, on the DDRNet-23 batch-32 3x3 stride-1 shapes (us, TFLOP/s).
  python tools/bench_whalo.py [--batch 32]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402

SHAPES = [(64, 256, 512, 64), (128, 128, 256, 128), (256, 128, 256, 128), (256, 64, 128, 256), (512, 32, 64, 512)]


def t_us(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / iters * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    assert ops.load()
    o = torch.ops.rtseg
    cl = torch.channels_last
    for cin, h, w, cout in SHAPES:
        x = torch.randn(a.batch, cin, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        dy = torch.randn(a.batch, cout, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        fl = 2.0 * a.batch * h * w * cin * cout * 9
        r = [o.conv_whalo_wgrad(x, dy, 3, 3, [1, 1], [1, 1], [1, 1], True, v) for v in (1, 2)]
        err = ((r[0] - r[1]).norm() / r[0].norm()).item()
        ts = [t_us(lambda v=v: o.conv_whalo_wgrad(x, dy, 3, 3, [1, 1], [1, 1], [1, 1], True, v)) for v in (1, 2)]
        print(f"{cin:4d}->{cout:4d} @ {h}x{w}: v1 {ts[0]:7.1f} us ({fl / ts[0] / 1e6:6.0f} TF/s)  "
              f"v2 {ts[1]:7.1f} us ({fl / ts[1] / 1e6:6.0f} TF/s)  rel diff {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
