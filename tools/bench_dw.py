"""Depth-wise conv forward (dwconv.hip) on the KD teacher's ASPP shapes and zoo shapes: time, achieved
HBM-equivalent bandwidth (input + output bytes once) and max error vs F.conv2d, per launch path.
Run twice (RTSEG_DW_CS=0 / 1, read at library load) for the A/B.
python tools/bench_dw.py [--iters 20]"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402

# (N, C, H, W, k, stride, dilation, stats)
SHAPES = [
    (16, 2048, 64, 128, 3, 1, 12, False),  # DeepLabV3+ ASPP separable convs at 1/16 (KD teacher)
    (16, 2048, 64, 128, 3, 1, 24, False),
    (16, 2048, 64, 128, 3, 1, 36, False),
    (16, 256, 256, 512, 3, 1, 1, False),   # DeepLabV3+ decoder separable conv at 1/4
    (16, 128, 128, 256, 3, 1, 1, True),    # DWConvBNAct (training, BN statistics epilogue)
    (16, 64, 256, 512, 3, 2, 1, True),
    (16, 32, 512, 1024, 3, 1, 2, True),
]


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
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    assert ops.load()
    r = torch.ops.rtseg
    tag = "cs" if os.environ.get("RTSEG_DW_CS", "1") != "0" else "base"
    for n, c, h, w, k, s, d, st in SHAPES:
        x = torch.randn(n, c, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wgt = torch.randn(c, 1, k, k, device="cuda") / k
        wt = wgt.reshape(c, k * k).t().contiguous()
        p = d * (k // 2)
        if st:
            fn = lambda: r.dw_conv_fwd_stats(x, wt, c, k, k, s, s, p, p, d, d)[0]  # noqa: E731
        else:
            fn = lambda: r.dw_conv_fwd(x, wt, None, c, k, k, s, s, p, p, d, d)  # noqa: E731
        y = fn()
        ref = F.conv2d(x.float(), wgt, None, s, p, d, c)
        err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
        us = timeit(fn, a.iters)
        gb = (x.numel() + y.numel()) * 2 / 1e9
        print(f"{tag:4s} N{n} C{c} {h}x{w} k{k} s{s} d{d}{' +stats' if st else ''}: {us:9.1f} us "
              f"{gb / us * 1e6 / 1e3:6.2f} TB/s  err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
