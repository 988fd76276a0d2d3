"""The KD teacher's ResNet stem (7 x 7 / 2, 3 -> 64, batch 16, 1024 x 2048, bf16) on MIOpen in each
memory layout (the channels-last pick measured 1.5 ms per call in the KD profile, profiles/r6_kd),
and the native conv_stem7.hip kernel (alone, and with the inference BN + ReLU epilogue).
python tools/bench_stem7.py"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                          "miopen_db"))


def timeit(fn, iters=10):
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
    torch.backends.cudnn.benchmark = True
    x = torch.randn(16, 3, 1024, 2048, device="cuda").to(torch.bfloat16)
    w = (torch.randn(64, 3, 7, 7, device="cuda") / 12).to(torch.bfloat16)
    xcl = x.contiguous(memory_format=torch.channels_last)
    wcl = w.contiguous(memory_format=torch.channels_last)
    ref = F.conv2d(x.float()[:1], w.float(), None, 2, 3)
    from realtime_semantic_segmentation_pytorch_amd import ops

    assert ops.load()
    wk = w.permute(0, 2, 3, 1).contiguous()
    ss = torch.cat([torch.ones(64), torch.zeros(64)]).cuda()
    for name, fn in [("rtseg conv_stem7", lambda: torch.ops.rtseg.conv_stem7(xcl, wk, [2, 2], None, 0)),
                     ("rtseg conv_stem7 + BN/ReLU", lambda: torch.ops.rtseg.conv_stem7(xcl, wk, [2, 2], ss, 1)),("nchw", lambda: F.conv2d(x, w, None, 2, 3)),
                     ("channels_last", lambda: F.conv2d(xcl, wcl, None, 2, 3)),
                     ("nchw + to channels_last", lambda: F.conv2d(xcl.contiguous(), w, None, 2, 3).contiguous(
                         memory_format=torch.channels_last))]:
        y = fn()
        err = (y[:1].float() - ref).abs().max().item() / ref.abs().max().item()
        print(f"{name:28s} {timeit(fn):9.1f} us  err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
