"""Channel-multiplier depth-wise conv (dwconv.hip) on BiSeNetV2's x6 gather-expansion shapes (batch
16, 1024x2048): forward + BN statistics, data gradient and weight gradient -- time, HBM-equivalent
bandwidth (each operand once) and error vs an fp32 reference.  Run twice for the A/B
(RTSEG_DW_WG_PAIR=0 RTSEG_DW_MT_CS=0 vs defaults; read at first launch).
python tools/bench_dw_mult.py [--iters 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402

# (N, Cin, H, W, mult, stride): the GE layers' DWConvBNAct(in, 6 in, 3, s) (bisenetv2.py GE)
SHAPES = [
    (16, 16, 256, 512, 6, 2),
    (16, 32, 128, 256, 6, 1),
    (16, 32, 128, 256, 6, 2),
    (16, 64, 64, 128, 6, 1),
    (16, 64, 64, 128, 6, 2),
    (16, 128, 32, 64, 6, 1),
    # plain depth-wise (multiplier 1): the GE layers' second DW and the stride-2 shortcut DW
    (16, 96, 128, 256, 1, 1),
    (16, 192, 64, 128, 1, 1),
    (16, 384, 32, 64, 1, 1),
    (16, 16, 256, 512, 1, 2),
    (16, 32, 128, 256, 1, 2),
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
    tag = "new" if os.environ.get("RTSEG_DW_MT_CS", "1") != "0" else "base"
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for n, c, h, w, m, s in SHAPES:
        co = c * m
        ho, wo = (h + 2 - 3) // s + 1, (w + 2 - 3) // s + 1
        x = torch.randn(n, c, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(n, co, ho, wo, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wgt = torch.randn(co, 1, 3, 3, device="cuda") / 3
        wt = wgt.reshape(co, 9).t().contiguous()
        gb = (x.numel() + dy.numel()) * 2 / 1e9
        cases = {
            "fwd": (lambda: r.dw_conv_fwd_stats(x, wt, co, 3, 3, s, s, 1, 1, 1, 1)[0],
                    lambda: torch.nn.functional.conv2d(x.float(), wgt, None, s, 1, 1, c)),
            "dgrad": (lambda: r.dw_conv_dgrad(dy, wt, c, h, w, 3, 3, s, s, 1, 1, 1, 1),
                      lambda: torch.nn.grad.conv2d_input(x.shape, wgt, dy.float(), s, 1, 1, c)),
            "wgrad": (lambda: r.dw_conv_wgrad(dy, x, 3, 3, s, s, 1, 1, 1, 1),
                      lambda: torch.nn.grad.conv2d_weight(x.float(), (co, 1, 3, 3), dy.float(), s, 1, 1, c)),
        }
        for name, (fn, ref_fn) in cases.items():
            got, ref = fn().float(), ref_fn()
            err = (got - ref).abs().max().item() / ref.abs().max().item()
            us = timeit(fn, a.iters)
            tot[name] += us
            print(f"{tag:4s} {name:5s} N{n} Cin{c} x{m} {h}x{w} s{s}: {us:8.1f} us {gb / us * 1e6 / 1e3:5.2f} TB/s  "
                  f"err {err:.1e}", flush=True)
    print(f"{tag:4s} total " + "  ".join(f"{k} {v:.1f} us" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
