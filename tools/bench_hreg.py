"""conv_hreg wave layouts (1: 8 waves x 2x2 tiles, 2: 4 waves x 2x4, 4: 8 waves x 1x4) against the
igemm gather kernel on DDRNet-23's 3 x 3 stride-1 shapes at batch 32, 1024 x 2048: forward with the
BN-statistics epilogue and data gradient.  One line per (shape, pass): us and TFLOP/s per kernel,
max error of each layout against igemm.
python tools/bench_hreg.py [--batch 32] [--iters 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402

# (Cin, H, W, Cout): conv input sizes
SHAPES = [(128, 128, 256, 128), (256, 64, 128, 256), (512, 32, 64, 512), (128, 64, 128, 128), (256, 32, 64, 256),
          (64, 128, 256, 128)]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    assert ops.load()
    r = torch.ops.rtseg
    cl = dict(memory_format=torch.channels_last)
    for cin, h, w, cout in SHAPES:
        n = a.batch
        x = torch.randn(n, cin, h, w, device="cuda").to(torch.bfloat16).contiguous(**cl)
        wt = (torch.randn(cout, cin, 3, 3, device="cuda") / (cin * 9) ** 0.5).to(torch.bfloat16)
        wk, wtr = wt.permute(0, 2, 3, 1).contiguous(), wt.permute(1, 2, 3, 0).contiguous()
        dy = torch.randn(n, cout, h, w, device="cuda").to(torch.bfloat16).contiguous(**cl)
        flop = 2.0 * n * h * w * cin * cout * 9
        passes = {
            "fwd+st": {"igemm": lambda: r.conv_igemm(x, wk, [1, 1], [1, 1], [1, 1], True, None, None, 0)[0]}
            | {f"hreg{k}": (lambda k=k: r.conv_hreg(x, wk, [1, 1], [1, 1], [1, 1], True, k)[0]) for k in (1, 2, 4, 5)},
        }
        if cin % 128 == 0:  # the dgrad produces Cin channels: % 128
            passes["dgrad"] = {"igemm": lambda: r.conv_igemm_dgrad(dy, wtr, list(x.shape), [1, 1], [1, 1], [1, 1])} | {
                f"hreg{k}": (lambda k=k: r.conv_hreg_dgrad(dy, wtr, list(x.shape), [1, 1], [1, 1], [1, 1], None, k))
                for k in (1, 2, 4, 5)}
        for pname, fns in passes.items():
            ref = fns["igemm"]().float()
            row = []
            for name, fn in fns.items():
                e = (fn().float() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
                us = timeit(fn, a.iters)
                row.append(f"{name} {us:8.1f} us {flop / us / 1e6:6.1f} TF err {e:.1e}")
            print(f"{cin:4d}x{h}x{w}->{cout:4d} {pname:6s} | " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
