#!/usr/bin/env python3
"""Where does a bf16-autocast inference forward leave bf16?  Every aten op of one eval forward
(the InferenceEngine's model form: bf16 weights, channels-last, autocast) is intercepted with a
TorchDispatchMode; ops that produce fp32 from bf16 inputs (casts, fp32-autocast ops) and every
copy are counted by (op, the innermost model source line).  Also counts MIOpen convs by
geometry, to spot the ones that fall back to naive kernels.

  python tools/probe_casts.py --models dfanet,espnetv2,fastscnn [--size 512x1024]
"""
from __future__ import annotations

import argparse
import collections
import copy
import os
import sys
import traceback

import torch
import torch.nn as nn
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.models import get_model  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.ops.act import _HipAct  # noqa: E402

PKG = "realtime_semantic_segmentation_pytorch_amd"


def _site():
    for fr in reversed(traceback.extract_stack()[:-3]):
        if PKG in fr.filename and "/ops/" not in fr.filename:
            return f"{fr.filename.split(PKG + '/')[-1]}:{fr.lineno} {fr.line.strip()[:60]}"
    return "?"


class Probe(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.hits = collections.Counter()
        self.convs = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func.overloadpacket.__name__)
        ins = [a for a in args if isinstance(a, torch.Tensor)]
        outs = out if isinstance(out, (tuple, list)) else [out]
        outs = [o for o in outs if isinstance(o, torch.Tensor)]
        if name in ("convolution", "cudnn_convolution", "miopen_convolution") and len(ins) >= 2:
            x, w = ins[0], ins[1]
            self.convs[(tuple(x.shape), tuple(w.shape), str(x.dtype)[6:], _site())] += 1
        up = any(i.dtype == torch.bfloat16 for i in ins) and any(o.dtype == torch.float32 for o in outs)
        if up or name in ("_to_copy", "copy_", "clone", "contiguous"):
            key = (name, "bf16->fp32" if up else "", _site())
            self.hits[key] += 1
        return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--models", default="dfanet,espnetv2,fastscnn")
    p.add_argument("--size", default="512x1024")
    a = p.parse_args()
    h, w = map(int, a.size.split("x"))
    assert ops.load()
    for key in a.models.split(","):
        c = BaseConfig()
        c.model, c.num_class = key, 19
        m = get_model(c).cuda().eval().to(memory_format=torch.channels_last)
        m = copy.deepcopy(m)
        for mod in m.modules():  # the InferenceEngine's weight cast (utils/inference.py)
            if isinstance(mod, (nn.Conv2d, nn.ConvTranspose2d, nn.Linear)) or (
                    isinstance(mod, nn.PReLU) and not isinstance(mod, _HipAct)):
                mod.to(torch.bfloat16)
        x = torch.randn(1, 3, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            ops.materialize(m(x))  # warm (autotune)
            probe = Probe()
            with probe:
                ops.materialize(m(x))
        print(f"== {key}: dtype round trips / copies per forward")
        for (name, kind, site), n in probe.hits.most_common(40):
            print(f"  {n:5d}  {name:14s} {kind:10s} {site}")
        print(f"== {key}: convolutions reaching aten (MIOpen) per forward")
        for (xs, ws, dt, site), n in probe.convs.most_common(40):
            print(f"  {n:5d}  x{xs} w{ws} {dt}  {site}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
