"""MFMA implicit-GEMM conv (``torch.ops.rtseg.conv_mfma``) vs MIOpen on the DDRNet-23 layer shapes.

Run on the GPU box:  python tools/bench_conv.py [--batch 16] [--iters 20]
Prints one line per shape: max-abs error vs F.conv2d (fp32 accumulate), times (us) and TFLOP/s of
MIOpen conv, conv_mfma, conv_mfma + BN-statistics epilogue, and MIOpen conv + the separate BN
statistics pass it replaces.
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                          "miopen_db"))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402

# (Cin, H, W, Cout, k, stride) at 1024x2048 input; H, W are the conv INPUT sizes
SHAPES = [
    (64, 256, 512, 64, 3, 1),
    (64, 256, 512, 128, 3, 2),
    (128, 128, 256, 128, 3, 1),
    (128, 128, 256, 256, 3, 2),
    (256, 64, 128, 256, 3, 1),
    (256, 64, 128, 512, 3, 2),
    (512, 32, 64, 512, 3, 1),
    (256, 64, 128, 128, 1, 1),
    (512, 16, 32, 1024, 1, 1),
    (128, 128, 256, 64, 1, 1),
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
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    assert ops.load()
    torch.backends.cudnn.benchmark = True
    dev = "cuda"
    print(f"{'shape':42s} {'err':>9s} {'miopen':>8s} {'mfma':>8s} {'mfma+st':>8s} {'mio+st':>8s}  TF(mio/mfma)")
    for cin, h, w, cout, k, s in SHAPES:
        n = a.batch
        torch.manual_seed(0)
        x = torch.randn(n, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, k, k, device=dev) * (1.0 / (cin * k * k) ** 0.5)).to(torch.bfloat16)
        wcl = wt.contiguous(memory_format=torch.channels_last)
        wk = wt.permute(0, 2, 3, 1).contiguous()
        p = k // 2
        y_ref = F.conv2d(x, wcl, None, s, p)
        y, _ = torch.ops.rtseg.conv_mfma(x, wk, [s, s], [p, p], [1, 1], False, None, None, 0)
        err = (y.float() - y_ref.float()).abs().max().item() / max(1e-6, y_ref.float().abs().max().item())
        t_mio = timeit(lambda: F.conv2d(x, wcl, None, s, p), a.iters)
        t_mf = timeit(lambda: torch.ops.rtseg.conv_mfma(x, wk, [s, s], [p, p], [1, 1], False, None, None, 0), a.iters)
        t_mfs = timeit(lambda: torch.ops.rtseg.conv_mfma(x, wk, [s, s], [p, p], [1, 1], True, None, None, 0), a.iters)
        t_mios = timeit(lambda: torch.ops.rtseg.bn_stats_sums(F.conv2d(x, wcl, None, s, p)), a.iters)
        ho, wo = y.shape[2], y.shape[3]
        flop = 2.0 * n * ho * wo * cout * cin * k * k
        tag = f"{n}x{cin}x{h}x{w} -> {cout} k{k} s{s}"
        print(f"{tag:42s} {err:9.2e} {t_mio:8.1f} {t_mf:8.1f} {t_mfs:8.1f} {t_mios:8.1f}  "
              f"{flop / t_mio / 1e6:6.0f}/{flop / t_mf / 1e6:6.0f}", flush=True)


if __name__ == "__main__":
    main()
