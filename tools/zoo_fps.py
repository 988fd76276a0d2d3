"""Whole-zoo inference FPS vs the reference's published RTX 2080 numbers.

The reference's only published performance figures are the FPS column of its
README model table (`README.md:133-172`, measured by `tools/test_speed.py` at
batch 1, 1024x512, fp32).  This tool measures every row of that table on one
MI355X with the same protocol -- batch 1, W x H = 1024 x 512, random input,
eval mode -- on the graph-captured engine (``utils/inference.py``), in fp32
(the reference's precision) and in bf16, and prints/writes one JSON line per
model plus a markdown table.

  python tools/zoo_fps.py --out gpurun_out/zoo_fps.jsonl [--only ddrnet,stdc]

Weights are random-init (no network); the architectures are the zoo's own.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.models import get_model  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.utils.inference import InferenceEngine  # noqa: E402

# (row label, model key, config overrides, README FPS on RTX 2080 at 1024x512 fp32) -- BASELINE.md
ROWS = [
    ("ADSCNet", "adscnet", {}, 89), ("AGLNet", "aglnet", {}, 61),
    ("BiSeNetv1", "bisenetv1", {}, 88), ("BiSeNetv2", "bisenetv2", {}, 142),
    ("CANet", "canet", {}, 76), ("CFPNet", "cfpnet", {}, 64), ("CGNet", "cgnet", {}, 157),
    ("ContextNet", "contextnet", {}, 80), ("DABNet", "dabnet", {}, 140),
    ("DDRNet-23-slim", "ddrnet", {"arch_type": "DDRNet-23-slim"}, 233),
    ("DFANet", "dfanet", {}, 60), ("EDANet", "edanet", {}, 125), ("ENet", "enet", {}, 140),
    ("ERFNet", "erfnet", {}, 60), ("ESNet", "esnet", {}, 66), ("ESPNet", "espnet", {}, 111),
    ("ESPNetv2", "espnetv2", {}, 101), ("FarseeNet", "farseenet", {}, 130),
    ("FastSCNN", "fastscnn", {}, 358), ("FDDWNet", "fddwnet", {}, 51), ("FPENet", "fpenet", {}, 90),
    ("FSSNet", "fssnet", {}, 121), ("ICNet", "icnet", {}, 102), ("LEDNet", "lednet", {}, 76),
    ("LinkNet", "linknet", {}, 106), ("Lite-HRNet", "lite_hrnet", {}, 30),
    ("LiteSeg", "liteseg", {}, 117), ("MiniNet", "mininet", {}, 254),
    ("MiniNetv2", "mininetv2", {}, 86),
    ("PP-LiteSeg-STDC1", "ppliteseg", {"encoder_type": "stdc1"}, 201),
    ("PP-LiteSeg-STDC2", "ppliteseg", {"encoder_type": "stdc2"}, 136),
    ("RegSeg", "regseg", {}, 104), ("SegNet", "segnet", {}, 14), ("ShelfNet", "shelfnet", {}, 110),
    ("SQNet", "sqnet", {}, 69), ("STDC1", "stdc", {"encoder_type": "stdc1"}, 163),
    ("STDC2", "stdc", {"encoder_type": "stdc2"}, 119), ("SwiftNet", "swiftnet", {}, 141),
]


def _fps(eng, x, seconds):
    for _ in range(3):
        eng(x)
    torch.cuda.synchronize()
    n, t0 = 0, time.perf_counter()
    while True:
        for _ in range(10):
            eng(x)
        n += 10
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return n / dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/zoo_fps.jsonl")
    ap.add_argument("--only", default="")
    ap.add_argument("--skip", default="")
    ap.add_argument("--seconds", type=float, default=0.5)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--benchmark", action="store_true",
                    help="MIOpen find mode (cudnn.benchmark); off by default: its exhaustive search "
                         "faulted the GPU on CFPNet's 1024x512 fp32 shapes")
    args = ap.parse_args()
    only = set(filter(None, args.only.split(",")))
    skip = set(filter(None, args.skip.split(",")))
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    torch.backends.cudnn.benchmark = args.benchmark
    x = torch.randn(1, 3, args.height, args.width, device="cuda")
    rows = []
    with open(args.out, "a") as f:
        for label, key, over, ref in ROWS:
            if only and key not in only and label not in only:
                continue
            if key in skip or label in skip:
                continue
            c = BaseConfig()
            c.model, c.num_class, c.use_aux, c.use_detail_head = key, 19, False, False
            c.encoder_weights = None
            for k, v in over.items():
                setattr(c, k, v)
            torch.manual_seed(0)
            rec = {"model": label, "key": key, "ref_fps_rtx2080": ref}
            print(f"[zoo_fps] {label} ...", flush=True)
            try:
                for name, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
                    eng = InferenceEngine(get_model(c), (1, 3, args.height, args.width), dtype=dt,
                                          use_graph=True, warmup=3)
                    rec[f"fps_{name}"] = round(_fps(eng, x, args.seconds), 1)
                    del eng
                rec["x_fp32"] = round(rec["fps_fp32"] / ref, 2)
                rec["x_bf16"] = round(rec["fps_bf16"] / ref, 2)
            except Exception as e:  # a model that cannot run is reported, not hidden
                rec["error"] = f"{type(e).__name__}: {e}"[:300]
            torch.cuda.empty_cache()
            rows.append(rec)
            f.write(json.dumps(rec) + "\n")
            f.flush()
            print(json.dumps(rec), flush=True)
    print("\n| Model | RTX 2080 FPS (README) | MI355X fp32 FPS | x | MI355X bf16 FPS | x |")
    print("|---|---|---|---|---|---|")
    for r in rows:
        if "error" in r:
            print(f"| {r['model']} | {r['ref_fps_rtx2080']} | error | | | |")
        else:
            print(f"| {r['model']} | {r['ref_fps_rtx2080']} | {r['fps_fp32']:.0f} | {r['x_fp32']:.2f} "
                  f"| {r['fps_bf16']:.0f} | {r['x_bf16']:.2f} |")


if __name__ == "__main__":
    main()
