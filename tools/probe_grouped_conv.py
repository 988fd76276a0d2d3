"""Grouped (non depth-wise) 3x3 convs at RegSeg's D-block shapes: MIOpen's grouped path vs the
same conv as one block-diagonal dense conv, forward + backward (bf16, channels-last, batch 8
at 1024x2048).  Prints ms per fwd+bwd for each formulation.

  python tools/probe_grouped_conv.py
"""
import time

import torch
import torch.nn.functional as F


def blockdiag(w, groups):
    cout, cg, kh, kw = w.shape
    mask = torch.zeros(cout, cg * groups, 1, 1, device=w.device, dtype=w.dtype)
    for g in range(groups):
        mask[g * (cout // groups):(g + 1) * (cout // groups), g * cg:(g + 1) * cg] = 1
    return w.repeat(1, groups, 1, 1) * mask


def run(n, c, h, w, groups, stride, dil, dense):
    x = torch.randn(n, c, h, w, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    x.requires_grad_(True)
    wt = torch.randn(c, c // groups, 3, 3, device="cuda", requires_grad=True)
    gy = None

    def step():
        nonlocal gy
        with torch.autocast("cuda", torch.bfloat16):
            if dense:
                y = F.conv2d(x, blockdiag(wt, groups), None, stride, dil, dil, 1)
            else:
                y = F.conv2d(x, wt, None, stride, dil, dil, groups)
        if gy is None:
            gy = torch.randn_like(y)
        torch.autograd.backward(y, gy)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    reps = 5
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    torch.backends.cudnn.benchmark = True
    shapes = [  # (n, c, h, w, groups, stride, dilation): RegSeg D-blocks at batch 8, 1024 x 2048
        (8, 48, 512, 1024, 3, 2, 1),
        (8, 128, 256, 512, 8, 2, 1),
        (8, 64, 128, 256, 4, 1, 1),
        (8, 256, 128, 256, 16, 2, 1),
        (8, 128, 64, 128, 8, 1, 2),
        (8, 128, 64, 128, 8, 1, 11),
        (8, 320, 64, 128, 20, 2, 5),
    ]
    for s in shapes:
        g = run(*s, dense=False)
        d = run(*s, dense=True)
        print(f"{s}: grouped {g:8.3f} ms  block-diag dense {d:8.3f} ms", flush=True)


if __name__ == "__main__":
    main()
