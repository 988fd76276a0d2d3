"""Inference (tools/test_speed.py protocol) under rocprofv3: DDRNet-23, batch 1, HIP graph.

  rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/profile_infer.py [--model ddrnet --arch DDRNet-23]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(ROOT, "miopen_db"))

import torch  # noqa: E402

from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.models import get_model  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.utils.inference import InferenceEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="ddrnet")
    ap.add_argument("--arch", default="DDRNet-23")
    ap.add_argument("--h", type=int, default=1024)
    ap.add_argument("--w", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--fp32", action="store_true")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    c = BaseConfig()
    c.model, c.num_class, c.use_aux = a.model, 19, a.model == "ddrnet"
    if a.model == "ddrnet":
        c.arch_type = a.arch
    m = get_model(c).cuda()
    eng = InferenceEngine(m, (1, 3, a.h, a.w), dtype=torch.float32 if a.fp32 else torch.bfloat16, warmup=5)
    x = torch.randn(1, 3, a.h, a.w, device="cuda")
    for _ in range(5):
        eng(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        eng(x)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    print(f"{a.model} {a.arch} {a.h}x{a.w} {'fp32' if a.fp32 else 'bf16'}: {dt * 1e3:.3f} ms/img  {1 / dt:.1f} FPS")


if __name__ == "__main__":
    main()
