#!/usr/bin/env python3
"""A/B of the conv_igemm epilogue store width (RTSEG_IGEMM_WIDE_STORE, read per launch): 8-byte
stores per channel group vs 16-byte stores of channel-group pairs exchanged across the half-waves
(v_permlane32_swap).  DDRNet-23 b32 shapes, forward (+ BN statistics) and data gradient, default
tile configuration, interleaved, best of 3 rounds; outputs compared bitwise.

  python tools/bench_igemm_wide.py [--batch 32]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402

# (cin, h, w, cout, k, stride)
SHAPES = [(128, 128, 256, 128, 3, 1), (256, 128, 256, 128, 3, 1), (256, 64, 128, 256, 3, 1), (512, 32, 64, 512, 3, 1),
          (64, 256, 512, 64, 3, 1), (64, 512, 1024, 64, 3, 2), (64, 256, 512, 128, 3, 2), (128, 128, 256, 256, 3, 2),
          (128, 128, 256, 64, 1, 1), (64, 128, 256, 128, 1, 1)]


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
    tot = {"0": 0.0, "1": 0.0}
    for cin, h, w, cout, k, s in SHAPES:
        p = (k - 1) // 2
        ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        x = torch.randn(a.batch, cin, h, w, device="cuda", dtype=torch.bfloat16).contiguous(**cl)
        wt = (torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).to(torch.bfloat16)
        wk = wt.permute(0, 2, 3, 1).contiguous()
        wtr = wt.permute(1, 2, 3, 0).contiguous()
        dy = torch.randn(a.batch, cout, ho, wo, device="cuda", dtype=torch.bfloat16).contiguous(**cl)
        st = [s, s]
        fns = {"fwd+st": lambda: r.conv_igemm(x, wk, st, [p, p], [1, 1], True, None, None, 0)[0],
               "fwd": lambda: r.conv_igemm(x, wk, st, [p, p], [1, 1], False, None, None, 0)[0],
               "dgrad": lambda: r.conv_igemm_dgrad(dy, wtr, list(x.shape), st, [p, p], [1, 1])}
        for name, fn in fns.items():
            best, outs = {}, {}
            for rnd in range(3):
                for wd in ("0", "1"):
                    os.environ["RTSEG_IGEMM_WIDE_STORE"] = wd
                    if rnd == 0:
                        outs[wd] = fn().clone()
                    best[wd] = min(best.get(wd, float("inf")), timeit(fn))
            for wd in best:
                tot[wd] += best[wd]
            print(f"{cin}->{cout} k{k} s{s} @ {h}x{w} {name:7s} 8B {best['0']:8.1f} us  16B {best['1']:8.1f} us "
                  f"({best['0'] / best['1']:.3f}x)  equal={torch.equal(outs['0'], outs['1'])}", flush=True)
        os.environ.pop("RTSEG_IGEMM_WIDE_STORE", None)
        del x, dy
    print(f"total 8B {tot['0']:.1f} us  16B {tot['1']:.1f} us ({tot['0'] / tot['1']:.3f}x)")


if __name__ == "__main__":
    main()
