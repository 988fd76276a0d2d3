"""1x1 convolution as a plain GEMM on channels-last [P, C] views (hipBLASLt via torch.mm) vs
MIOpen F.conv2d, forward + backward (dgrad + wgrad), bf16, DDRNet-23 1x1 shapes at batch 32.

Run on the GPU box: python tools/bench_1x1.py [--batch 32]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                          "miopen_db"))

SHAPES = [(256, 64, 128, 128), (512, 32, 64, 128), (128, 128, 256, 64), (64, 256, 512, 128),
          (512, 16, 32, 1024), (1024, 16, 32, 256), (128, 128, 256, 256), (256, 128, 256, 19)]


def graph_time(fn, iters=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    print(f"{'shape':34s} {'mio_f':>7s} {'gemm_f':>7s} {'mio_dg':>7s} {'gemm_dg':>7s} {'mio_wg':>7s} {'gemm_wg':>7s}  (us)")
    for cin, h, w, cout in SHAPES:
        n = a.batch
        x = torch.randn(n, cin, h, w, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = torch.randn(cout, cin, 1, 1, device="cuda", dtype=torch.bfloat16) * 0.05
        gy = torch.randn(n, cout, h, w, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x2, g2, w2 = x.permute(0, 2, 3, 1).reshape(-1, cin), gy.permute(0, 2, 3, 1).reshape(-1, cout), wt.view(cout, cin)
        t = [graph_time(lambda: F.conv2d(x, wt)), graph_time(lambda: torch.mm(x2, w2.t())),
             graph_time(lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, [1, 1], [0, 0], [1, 1], False,
                                                                    [0, 0], 1, [True, False, False])),
             graph_time(lambda: torch.mm(g2, w2)),
             graph_time(lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, [1, 1], [0, 0], [1, 1], False,
                                                                    [0, 0], 1, [False, True, False])),
             graph_time(lambda: torch.mm(g2.t(), x2))]
        print(f"{n}x{cin}x{h}x{w} -> {cout}".ljust(34) + " ".join(f"{v:7.1f}" for v in t), flush=True)


if __name__ == "__main__":
    main()
