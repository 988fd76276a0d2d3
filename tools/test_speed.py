"""Inference FPS (parity: reference tools/test_speed.py:9-62).

Same protocol -- batch 1, W x H = 2048 x 1024 scaled by ``--ratio`` (default
0.5 like the reference), 10 warm-up forwards, an adaptive iteration count for
~6 s of timing -- measured on the graph-captured engine (``--no-graph`` for
eager), in bf16 (``--fp32`` for fp32) and channels-last.

  python tools/test_speed.py --model ddrnet --arch_type DDRNet-23 --ratio 1.0
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd.configs import MyConfig, load_parser  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.models import get_model  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.utils.inference import InferenceEngine  # noqa: E402


def _pop_flag(argv, name, has_value=False, default=None):
    if name not in argv:
        return default
    i = argv.index(name)
    if has_value:
        v = argv[i + 1]
        del argv[i:i + 2]
        return v
    del argv[i]
    return True


def test_model_speed(config, ratio=0.5, imgw=2048, imgh=1024, iterations=None, dtype=torch.bfloat16,
                     use_graph=True):
    if ratio != 1.0:
        if ratio <= 0:
            raise AssertionError("Ratio should be larger than 0.\n")
        imgw, imgh = int(imgw * ratio), int(imgh * ratio)
    if config.model in ("ddrnet", "bisenetv2", "stdc", "pp_liteseg", "ppliteseg"):
        # shapes where the naive solvers only slow the find down; elsewhere they are the
        # fallback for degenerate dilated geometries (see the package docstring)
        os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
        # MIOpen find mode only on the shapes it has been verified on: its exhaustive search
        # faulted the GPU on CFPNet's 1024x512 fp32 convolutions (tools/zoo_fps.py)
        torch.backends.cudnn.benchmark = True
    model = get_model(config)
    print("\n=========Speed Testing=========")
    print(f"Model: {config.model}\nEncoder: {config.encoder}\nDecoder: {config.decoder}")
    print(f"Size (W, H): {imgw}, {imgh}  dtype: {dtype}  graph: {use_graph}")
    eng = InferenceEngine(model, (1, 3, imgh, imgw), dtype=dtype, use_graph=use_graph, warmup=10)
    x = torch.randn(1, 3, imgh, imgw, device="cuda")
    if iterations is None:
        iterations, elapsed = 100, 0.0
        while elapsed < 1:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iterations):
                eng(x)
            torch.cuda.synchronize()
            elapsed = time.perf_counter() - t0
            iterations *= 2
        iterations = int(iterations / 2 / elapsed * 6)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iterations):
        eng(x)
    torch.cuda.synchronize()
    latency = (time.perf_counter() - t0) / iterations * 1000
    fps = 1000 / latency
    print(f"FPS: {fps}\n")
    return fps


if __name__ == "__main__":
    argv = sys.argv[1:]
    ratio = float(_pop_flag(argv, "--ratio", True, 0.5))
    fp32 = _pop_flag(argv, "--fp32", default=False)
    no_graph = _pop_flag(argv, "--no-graph", default=False)
    config = load_parser(MyConfig(), argv)
    test_model_speed(config, ratio=ratio, dtype=torch.float32 if fp32 else torch.bfloat16, use_graph=not no_graph)
