"""Run one conv kernel variant repeatedly (for rocprofv3 --pmc passes).

python tools/conv_probe.py --kind halo|igemm|halo_dg|igemm_dg|wgrad|wres|wres_dg|whalo --shape CIN,H,W,COUT [--batch 32] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="halo")
    ap.add_argument("--shape", default="128,128,256,128")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--stats", action="store_true")
    a = ap.parse_args()
    assert ops.load()
    cin, h, w, cout = (int(v) for v in a.shape.split(","))
    x = torch.randn(a.batch, cin, h, w, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    wt = (torch.randn(cout, cin, 3, 3, device="cuda") / (cin * 9) ** 0.5).to(torch.bfloat16)
    wk = wt.permute(0, 2, 3, 1).contiguous()
    wtr = wt.permute(1, 2, 3, 0).contiguous()
    dy = torch.randn(a.batch, cout, h, w, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    r = torch.ops.rtseg
    fns = {
        "halo": lambda: r.conv_halo(x, wk, [1, 1], [1, 1], [1, 1], a.stats, None, None, 0),
        "igemm": lambda: r.conv_igemm(x, wk, [1, 1], [1, 1], [1, 1], a.stats, None, None, 0),
        "halo_dg": lambda: r.conv_halo_dgrad(dy, wtr, list(x.shape), [1, 1], [1, 1], [1, 1]),
        "igemm_dg": lambda: r.conv_igemm_dgrad(dy, wtr, list(x.shape), [1, 1], [1, 1], [1, 1]),
        "wgrad": lambda: r.conv_igemm_wgrad(x, dy, 3, 3, [1, 1], [1, 1], [1, 1]),
        "wres": lambda: r.conv_wres(x, wk, [1, 1], [1, 1], [1, 1], a.stats),
        "wres_dg": lambda: r.conv_wres_dgrad(dy, wtr, list(x.shape), [1, 1], [1, 1], [1, 1]),
        "whalo": lambda: r.conv_whalo_wgrad(x, dy, 3, 3, [1, 1], [1, 1], [1, 1]),
        "whalo2": lambda: r.conv_whalo_wgrad(x, dy, 3, 3, [1, 1], [1, 1], [1, 1], False, 2),
        "hreg": lambda: r.conv_hreg(x, wk, [1, 1], [1, 1], [1, 1], a.stats),
        "hreg_dg": lambda: r.conv_hreg_dgrad(dy, wtr, list(x.shape), [1, 1], [1, 1], [1, 1]),
        "hreg2": lambda: r.conv_hreg(x, wk, [1, 1], [1, 1], [1, 1], a.stats, 2),
        "hreg2_dg": lambda: r.conv_hreg_dgrad(dy, wtr, list(x.shape), [1, 1], [1, 1], [1, 1], None, 2),
        "hreg4": lambda: r.conv_hreg(x, wk, [1, 1], [1, 1], [1, 1], a.stats, 4),
        "hreg4_dg": lambda: r.conv_hreg_dgrad(dy, wtr, list(x.shape), [1, 1], [1, 1], [1, 1], None, 4),
        "hreg5": lambda: r.conv_hreg(x, wk, [1, 1], [1, 1], [1, 1], a.stats, 5),
        "hreg5_dg": lambda: r.conv_hreg_dgrad(dy, wtr, list(x.shape), [1, 1], [1, 1], [1, 1], None, 5),
    }
    if a.kind.startswith("stem"):  # the 3-channel stem at DDRNet-23's geometry (cin = 3, stride 2)
        xs = torch.randn(a.batch, 3, h, w, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        ws = (torch.randn(cout, 3, 3, 3, device="cuda") * 0.2).to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
        ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        dys = torch.randn(a.batch, cout, ho, wo, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        ss = torch.cat([torch.ones(cout), torch.zeros(cout)]).cuda()
        fns["stem_stats"] = lambda: r.conv_stem(xs, ws, [2, 2], [1, 1], [1, 1], True)
        fns["stem_nostore"] = lambda: r.conv_stem(xs, ws, [2, 2], [1, 1], [1, 1], True, False)
        fns["stem_apply"] = lambda: r.conv_stem_bn_act(xs, ws, [2, 2], [1, 1], [1, 1], ss, 1)
        fns["stem_wgrad"] = lambda: r.conv_stem_wgrad(xs, dys, 3, 3, [2, 2], [1, 1], [1, 1], True)
    fn = fns[a.kind]
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    print("done", a.kind, a.shape, flush=True)


if __name__ == "__main__":
    main()
