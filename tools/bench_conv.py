"""Hand-written MFMA conv kernels vs MIOpen on the DDRNet-23 layer shapes: forward, data gradient
and weight gradient.

Run on the GPU box:  python tools/bench_conv.py [--batch 32] [--iters 20] [--only fwd,dgrad,wgrad]
One line per shape and pass: relative max error vs MIOpen, time (us) of MIOpen and of ours,
TFLOP/s of both.  Ours: ``conv_igemm`` (+ its BN-statistics epilogue, ``fwd+st``),
``conv_igemm_dgrad``, ``conv_igemm_wgrad``, and for stride-1 3x3 shapes the halo-tiled
``conv_halo`` (``halo``, ``halo+st``) / ``conv_halo_dgrad`` (``halo_dg``), and where the conv sums
over 64 channels the weights-resident ``conv_wres`` (``wres``, ``wres+st``, ``wres_dg``); MIOpen: ``F.conv2d`` / ``aten.convolution_backward``
(MIOpen find mode, i.e. its best solver per shape).
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


def relerr(a, b):
    return (a.float() - b.float()).abs().max().item() / max(1e-6, b.float().abs().max().item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="fwd,dgrad,wgrad")
    ap.add_argument("--cfgs", default="", help="comma list of RTSEG_IGEMM_CFG tile configs to sweep (fwd/dgrad)")
    ap.add_argument("--shapes", default="", help="comma list of shape indices")
    ap.add_argument("--wcfgs", default="", help="comma list of RTSEG_WGRAD_CFG configs to sweep (wgrad)")
    a = ap.parse_args()
    passes = set(a.only.split(","))
    assert ops.load()
    torch.backends.cudnn.benchmark = True
    dev = "cuda"
    print(f"{'shape':34s} {'pass':7s} {'err':>9s} {'miopen':>8s} {'ours':>8s}  TF(mio/ours)  speedup", flush=True)
    conv_bw = torch.ops.aten.convolution_backward
    cfgs = [c for c in a.cfgs.split(",") if c != ""] or [None]
    shapes = [SHAPES[int(i)] for i in a.shapes.split(",")] if a.shapes else SHAPES
    for cin, h, w, cout, k, s in shapes:
        n = a.batch
        torch.manual_seed(0)
        x = torch.randn(n, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, k, k, device=dev) * (1.0 / (cin * k * k) ** 0.5)).to(torch.bfloat16)
        wcl = wt.contiguous(memory_format=torch.channels_last)
        wk = wt.permute(0, 2, 3, 1).contiguous()
        wtr = wt.permute(1, 2, 3, 0).contiguous()
        p = k // 2
        y_ref = F.conv2d(x, wcl, None, s, p)
        ho, wo = y_ref.shape[2], y_ref.shape[3]
        flop = 2.0 * n * ho * wo * cout * cin * k * k
        dy = torch.randn_like(y_ref).contiguous(memory_format=torch.channels_last)
        tag = f"{n}x{cin}x{h}x{w}->{cout} k{k}s{s}"
        halo = s == 1 and k == 3 and cin % 64 == 0 and cout % 64 == 0 and os.environ.get("RTSEG_CONV_HALO") != "0"
        wres = s == 1 and k == 3 and os.environ.get("RTSEG_CONV_WRES") != "0"
        rows = []
        for cfg in cfgs:
            sfx = "" if cfg is None else f"@{cfg}"
            if cfg is not None:
                os.environ["RTSEG_IGEMM_CFG"] = cfg
            if "fwd" in passes:
                y, _ = torch.ops.rtseg.conv_igemm(x, wk, [s, s], [p, p], [1, 1], False, None, None, 0)
                t_m = timeit(lambda: F.conv2d(x, wcl, None, s, p), a.iters)
                t_o = timeit(lambda: torch.ops.rtseg.conv_igemm(x, wk, [s, s], [p, p], [1, 1], False, None, None, 0),
                             a.iters)
                rows.append(("fwd" + sfx, relerr(y, y_ref), t_m, t_o))
                if cfg is None:
                    t_os = timeit(lambda: torch.ops.rtseg.conv_igemm(x, wk, [s, s], [p, p], [1, 1], True, None, None,
                                                                     0), a.iters)
                    rows.append(("fwd+st", 0.0, t_m, t_os))
                    if halo:  # the halo-tiled kernel (conv_halo.hip) on the same shape
                        yh, _ = torch.ops.rtseg.conv_halo(x, wk, [s, s], [p, p], [1, 1], False, None, None, 0)
                        t_h = timeit(lambda: torch.ops.rtseg.conv_halo(x, wk, [s, s], [p, p], [1, 1], False, None,
                                                                       None, 0), a.iters)
                        rows.append(("halo", relerr(yh, y_ref), t_m, t_h))
                        t_hs = timeit(lambda: torch.ops.rtseg.conv_halo(x, wk, [s, s], [p, p], [1, 1], True, None,
                                                                        None, 0), a.iters)
                        rows.append(("halo+st", 0.0, t_m, t_hs))
                    if wres and cin % 64 == 0 and cout % 128 == 0:  # register-weight halo kernel (conv_hreg.hip)
                        yg, _ = torch.ops.rtseg.conv_hreg(x, wk, [s, s], [p, p], [1, 1], False)
                        t_g = timeit(lambda: torch.ops.rtseg.conv_hreg(x, wk, [s, s], [p, p], [1, 1], False), a.iters)
                        rows.append(("hreg", relerr(yg, y_ref), t_m, t_g))
                        t_gs = timeit(lambda: torch.ops.rtseg.conv_hreg(x, wk, [s, s], [p, p], [1, 1], True), a.iters)
                        rows.append(("hreg+st", 0.0, t_m, t_gs))
                        yg, _ = torch.ops.rtseg.conv_hreg(x, wk, [s, s], [p, p], [1, 1], False, 2)
                        t_g = timeit(lambda: torch.ops.rtseg.conv_hreg(x, wk, [s, s], [p, p], [1, 1], False, 2), a.iters)
                        rows.append(("hreg2", relerr(yg, y_ref), t_m, t_g))
                        t_gs = timeit(lambda: torch.ops.rtseg.conv_hreg(x, wk, [s, s], [p, p], [1, 1], True, 2), a.iters)
                        rows.append(("hreg2+st", 0.0, t_m, t_gs))
                    if wres and cin == 64:  # the weights-resident halo kernel (conv_wres.hip)
                        yw, _ = torch.ops.rtseg.conv_wres(x, wk, [s, s], [p, p], [1, 1], False)
                        t_w = timeit(lambda: torch.ops.rtseg.conv_wres(x, wk, [s, s], [p, p], [1, 1], False), a.iters)
                        rows.append(("wres", relerr(yw, y_ref), t_m, t_w))
                        t_ws = timeit(lambda: torch.ops.rtseg.conv_wres(x, wk, [s, s], [p, p], [1, 1], True), a.iters)
                        rows.append(("wres+st", 0.0, t_m, t_ws))
            if "dgrad" in passes:
                dx_ref = conv_bw(dy, x, wcl, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [True, False, False])[0]
                dx = torch.ops.rtseg.conv_igemm_dgrad(dy, wtr, list(x.shape), [s, s], [p, p], [1, 1])
                t_m = timeit(lambda: conv_bw(dy, x, wcl, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                             [True, False, False]), a.iters)
                t_o = timeit(lambda: torch.ops.rtseg.conv_igemm_dgrad(dy, wtr, list(x.shape), [s, s], [p, p], [1, 1]),
                             a.iters)
                rows.append(("dgrad" + sfx, relerr(dx, dx_ref), t_m, t_o))
                if halo and cfg is None:
                    dxh = torch.ops.rtseg.conv_halo_dgrad(dy, wtr, list(x.shape), [s, s], [p, p], [1, 1])
                    t_h = timeit(lambda: torch.ops.rtseg.conv_halo_dgrad(dy, wtr, list(x.shape), [s, s], [p, p],
                                                                         [1, 1]), a.iters)
                    rows.append(("halo_dg", relerr(dxh, dx_ref), t_m, t_h))
                if wres and cout % 64 == 0 and cin % 128 == 0 and cfg is None:
                    dxg = torch.ops.rtseg.conv_hreg_dgrad(dy, wtr, list(x.shape), [s, s], [p, p], [1, 1])
                    t_g = timeit(lambda: torch.ops.rtseg.conv_hreg_dgrad(dy, wtr, list(x.shape), [s, s], [p, p],
                                                                         [1, 1]), a.iters)
                    rows.append(("hreg_dg", relerr(dxg, dx_ref), t_m, t_g))
                    dxg = torch.ops.rtseg.conv_hreg_dgrad(dy, wtr, list(x.shape), [s, s], [p, p], [1, 1], None, 2)
                    t_g = timeit(lambda: torch.ops.rtseg.conv_hreg_dgrad(dy, wtr, list(x.shape), [s, s], [p, p],
                                                                         [1, 1], None, 2), a.iters)
                    rows.append(("hreg2_dg", relerr(dxg, dx_ref), t_m, t_g))
                if wres and cout == 64 and cfg is None:
                    dxw = torch.ops.rtseg.conv_wres_dgrad(dy, wtr, list(x.shape), [s, s], [p, p], [1, 1])
                    t_w = timeit(lambda: torch.ops.rtseg.conv_wres_dgrad(dy, wtr, list(x.shape), [s, s], [p, p],
                                                                         [1, 1]), a.iters)
                    rows.append(("wres_dg", relerr(dxw, dx_ref), t_m, t_w))
        os.environ.pop("RTSEG_IGEMM_CFG", None)
        if "wgrad" in passes:
            dw_ref = conv_bw(dy, x, wcl, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [False, True, False])[1]
            t_m = timeit(lambda: conv_bw(dy, x, wcl, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                         [False, True, False]), a.iters)
            for wc in [c for c in a.wcfgs.split(",") if c != ""] or [None]:
                if wc is not None:
                    os.environ["RTSEG_WGRAD_CFG"] = wc
                dw = torch.ops.rtseg.conv_igemm_wgrad(x, dy, k, k, [s, s], [p, p], [1, 1])
                t_o = timeit(lambda: torch.ops.rtseg.conv_igemm_wgrad(x, dy, k, k, [s, s], [p, p], [1, 1]), a.iters)
                rows.append(("wgrad" + ("" if wc is None else f"@{wc}"), relerr(dw, dw_ref), t_m, t_o))
            os.environ.pop("RTSEG_WGRAD_CFG", None)
            if s == 1 and k == 3 and cin % 64 == 0 and cout % 64 == 0:  # halo-tiled wgrad (conv_whalo.hip)
                dwh = torch.ops.rtseg.conv_whalo_wgrad(x, dy, k, k, [s, s], [p, p], [1, 1])
                t_h = timeit(lambda: torch.ops.rtseg.conv_whalo_wgrad(x, dy, k, k, [s, s], [p, p], [1, 1]), a.iters)
                rows.append(("whalo", relerr(dwh, dw_ref), t_m, t_h))
        for name, err, t_m, t_o in rows:
            print(f"{tag:34s} {name:9s} {err:9.2e} {t_m:8.1f} {t_o:8.1f}  {flop / t_m / 1e6:5.0f}/{flop / t_o / 1e6:5.0f}"
                  f"   {t_m / t_o:5.2f}x", flush=True)
        del x, dy, y_ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
