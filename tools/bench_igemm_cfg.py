#!/usr/bin/env python3
"""Time every conv_igemm tile configuration (csrc/kernels/conv_igemm.hip kCfgs, forced through
RTSEG_IGEMM_CFG, read per launch) on the DDRNet-23 b32 3 x 3 shapes, forward (+ BN statistics)
and data gradient, next to the hreg / wres kernels the autotuner picks for some of them.

  python tools/bench_igemm_cfg.py [--batch 32]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402

# (cin, h, w, cout, stride)
SHAPES = [(128, 128, 256, 128, 1), (256, 128, 256, 128, 1), (256, 64, 128, 256, 1), (512, 32, 64, 512, 1),
          (64, 256, 512, 64, 1), (64, 256, 512, 128, 2), (128, 128, 256, 256, 2), (256, 64, 128, 512, 2)]


def timeit(fn, reps=10):
    try:
        fn()
    except RuntimeError:  # a kernel that does not take this geometry
        return float("nan")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    assert ops.load()
    r = torch.ops.rtseg
    for cin, h, w, cout, s in SHAPES:
        x = torch.randn(a.batch, cin, h, w, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, 3, 3, device="cuda") / (cin * 9) ** 0.5).to(torch.bfloat16)
        wk = wt.permute(0, 2, 3, 1).contiguous()
        wtr = wt.permute(1, 2, 3, 0).contiguous()
        ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
        dy = torch.randn(a.batch, cout, ho, wo, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        flop = 2.0 * a.batch * ho * wo * cout * cin * 9
        st = [s, s]
        row = {}
        for cfg in range(5):
            os.environ["RTSEG_IGEMM_CFG"] = str(cfg)
            row[f"fwd c{cfg}"] = timeit(lambda: r.conv_igemm(x, wk, st, [1, 1], [1, 1], True, None, None, 0))
            if cin % 8 == 0 and cout % 64 == 0:
                row[f"dg c{cfg}"] = timeit(lambda: r.conv_igemm_dgrad(dy, wtr, list(x.shape), st, [1, 1], [1, 1]))
        os.environ.pop("RTSEG_IGEMM_CFG", None)
        if s == 1:
            for v in (1, 2):
                row[f"fwd hreg{v}"] = timeit(lambda: r.conv_hreg(x, wk, st, [1, 1], [1, 1], True, v))
                row[f"dg hreg{v}"] = timeit(
                    lambda: r.conv_hreg_dgrad(dy, wtr, list(x.shape), st, [1, 1], [1, 1], None, v))
            row["fwd wres"] = timeit(lambda: r.conv_wres(x, wk, st, [1, 1], [1, 1], True))
            row["dg wres"] = timeit(lambda: r.conv_wres_dgrad(dy, wtr, list(x.shape), st, [1, 1], [1, 1]))
        print(f"== {cin}->{cout} @ {h}x{w} s{s}  ({flop / 1e9:.0f} GFLOP)")
        for k, t in row.items():
            print(f"   {k:10s} {t:8.1f} us  {flop / t / 1e6:7.0f} TF/s")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
