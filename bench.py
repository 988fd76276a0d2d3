#!/usr/bin/env python3
"""Headline benchmark: DDRNet-23 training throughput at 1024x2048, 19 classes.

BASELINE.json metric: "train images/sec (whole node) + single-GPU inference
FPS, DDRNet-23 1024x2048 19-class".  One process per GPU (torchrun), RCCL
all-reduce for N>1.  The timed region is the production training step of
``SegTrainer.train_step`` -- forward (bf16 autocast, channels-last), OHEM loss on
the main head + aux head (fused HIP kernels), backward, DDP gradient
all-reduce, SGD step, OneCycle LR step and EMA update -- on synthetic
device-resident batches (random-init weights; no datasets/checkpoints here).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
  torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  ``value`` = images/s over all ranks (weak
scaling: B images per GPU per step); ``extra.infer_fps_*`` are single-GPU
eval-mode FPS numbers for the same model at 1024x2048, batch 1.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

_ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, _ROOT)
# MIOpen find mode without the naive solvers + the in-tree find database: the SAME settings
# SegTrainer applies (utils/runtime.py), so the bench measures what `main.py --train` runs.
from realtime_semantic_segmentation_pytorch_amd.utils.runtime import configure_backend  # noqa: E402

import torch
import torch.distributed as dist

from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig  # noqa: E402


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=32, help="images per GPU per step (288 GB HBM: 27 GB at 32)")
    p.add_argument("--height", type=int, default=1024)
    p.add_argument("--width", type=int, default=2048)
    p.add_argument("--model", default="ddrnet", help="registry key (ddrnet | bisenetv2 | stdc | ...)")
    p.add_argument("--arch", default="DDRNet-23", help="DDRNet arch_type / STDC+PP-LiteSeg encoder_type")
    p.add_argument("--detail-head", action="store_true", help="STDC: detail head instead of aux heads")
    p.add_argument("--kd", action="store_true",
                   help="knowledge distillation from an SMP DeepLabV3+/ResNet-101 teacher (random init)")
    p.add_argument("--no-infer", action="store_true", help="skip the inference-FPS measurement")
    p.add_argument("--graph-step", action="store_true",
                   help="replay forward+loss+backward from one captured HIP graph (SegTrainer.graph_step)")
    p.add_argument("--fp32", action="store_true", help="disable bf16 autocast (diagnostic)")
    p.add_argument("--no-fused-loss", action="store_true")
    p.add_argument("--nchw", action="store_true")
    p.add_argument("--profile-steps", type=int, default=0)
    p.add_argument("--cudnn-benchmark", choices=("auto", "on", "off"), default="auto",
                   help="MIOpen find mode for the convs left on MIOpen.  auto: on only at a recorded "
                        "config (FIND_RECORDED: the in-tree miopen_db/ holds its find results), so a new "
                        "batch / resolution never starts MIOpen's exhaustive solver search")
    p.add_argument("--no-cudnn-benchmark", action="store_true", help="same as --cudnn-benchmark off")
    return p.parse_args()


# (model, arch, batch, height, width) whose MIOpen find results are in miopen_db/ (the headline
# config and the BASELINE configs 3-4 at their bench batches)
FIND_RECORDED = {("ddrnet", "DDRNet-23", 32, 1024, 2048), ("bisenetv2", None, 16, 1024, 2048),
                 ("stdc", "stdc2", 16, 1024, 2048)}


def find_mode(a) -> bool:
    if a.no_cudnn_benchmark or a.cudnn_benchmark == "off":
        return False
    if a.cudnn_benchmark == "on":
        return True
    arch = a.arch if a.model in ("ddrnet", "stdc", "ppliteseg") else None
    return (a.model, arch, a.batch, a.height, a.width) in FIND_RECORDED


def make_config(a, world):
    c = BaseConfig()
    c.dataset = "cityscapes"
    c.num_class = 19
    c.model = a.model
    if a.model == "ddrnet":
        c.arch_type = a.arch
    elif a.model in ("stdc", "ppliteseg"):
        c.encoder_type = a.arch if a.arch.startswith("stdc") else "stdc2"
    c.use_detail_head = bool(a.detail_head)
    c.use_aux = a.model in ("ddrnet", "bisenetv2", "icnet", "stdc") and not a.detail_head
    c.loss_type = "ohem"
    c.optimizer_type = "sgd"
    c.train_bs = a.batch
    c.amp_training = not a.fp32
    c.amp_dtype = "bf16"
    c.channels_last = not a.nchw
    c.fused_loss = not a.no_fused_loss
    c.synthetic_data = True
    c.synthetic_size = (a.height, a.width)
    c.synthetic_len = a.batch * world * (a.steps + a.warmup + 8)
    c.total_epoch = 4
    c.crop_size = a.height
    c.crop_h, c.crop_w = a.height, a.width
    c.base_workers = 0
    c.save_ckpt = False
    c.use_tb = False
    c.load_ckpt = False
    c.save_dir = os.environ.get("RTSEG_BENCH_DIR", "/tmp/rtseg_bench")
    if a.kd:  # BASELINE config 5: DeepLabv3+/ResNet-101 teacher -> student, Hinton KL (T=4)
        c.kd_training = True
        c.teacher_model, c.teacher_encoder, c.teacher_decoder = "smp", "resnet101", "deeplabv3p"
        c.teacher_random_init = True
        c.kd_teacher_graph = os.environ.get("RTSEG_KD_EAGER", "0") != "1"  # A/B: eager teacher
    c.hip_activations = os.environ.get("RTSEG_DISABLE_ACT", "0") != "1"  # A/B: torch activations
    c.graph_step = bool(a.graph_step) and world == 1
    c.is_testing = False
    c.use_ema = True
    # a hung or dead rank fails the run within 5 minutes (parallel/ddp.py pg_timeout_s): the first
    # step's autotuning takes < 1 minute on every rank alike
    c.pg_timeout_s = 300
    return c


@torch.no_grad()
def infer_fps(model, h, w, dtype, channels_last, iters=50, warm=10):
    """tools/test_speed.py protocol (batch 1, eval) on the HIP-graph inference engine."""
    from realtime_semantic_segmentation_pytorch_amd.utils.inference import InferenceEngine

    eng = InferenceEngine(model, (1, 3, h, w), dtype=dtype, channels_last=channels_last, warmup=warm)
    x = torch.randn(1, 3, h, w, device="cuda")
    for _ in range(3):
        eng(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        eng(x)
    torch.cuda.synchronize()
    fps = iters / (time.perf_counter() - t0)
    del eng
    return fps


README_FPS_DDRNET23_SLIM = 233.0  # reference README.md:144 (RTX 2080, fp32, 1024x512, batch 1)


def _heartbeat(period=30.0):
    """stderr line every `period` s (MIOpen find on a fresh box can be silent for minutes)."""
    import threading

    stop = threading.Event()
    t0 = time.perf_counter()

    def run():
        while not stop.wait(period):
            print(f"[bench] alive {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()
    return stop


def main():
    a = parse()
    hb = _heartbeat()
    if os.environ.get("RTSEG_STACK_DUMP"):  # diagnose a stuck step: Python stacks every N s
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["RTSEG_STACK_DUMP"]), repeat=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and "LOCAL_RANK" not in os.environ:
        raise SystemExit("N>1 must be launched with torchrun (one process per GPU)")
    if a.gpus != world:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    if world == 1:
        os.environ.pop("LOCAL_RANK", None)

    from realtime_semantic_segmentation_pytorch_amd import ops
    from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer
    from realtime_semantic_segmentation_pytorch_amd.datasets import DeviceBatches
    from realtime_semantic_segmentation_pytorch_amd.parallel import barrier, de_parallel

    cfg = make_config(a, world)
    cfg.cudnn_benchmark = find_mode(a)
    configure_backend(cfg.cudnn_benchmark, model=cfg.model, exclude_naive=True)
    ops.load()
    trainer = SegTrainer(cfg)
    trainer.parallel_model(cfg)
    trainer.model.train()
    rank = dist.get_rank() if dist.is_initialized() else 0
    dev = trainer.device
    data = DeviceBatches(a.batch, (a.height, a.width), cfg.num_class, cfg.ignore_index, device=dev,
                         pool=2, channels_last=cfg.channels_last, seed=1234 + rank)

    def step():
        imgs, masks = data.next()
        return trainer.train_step(imgs, masks)

    t_warm = time.perf_counter()
    for i in range(a.warmup):
        t_w = time.perf_counter()
        step()
        if rank == 0:
            torch.cuda.synchronize()
            print(f"[bench] warm-up step {i + 1}/{a.warmup}: {time.perf_counter() - t_w:.2f} s",
                  file=sys.stderr, flush=True)

    def sync_all():
        torch.cuda.synchronize()
        if dist.is_initialized():
            barrier()
        torch.cuda.synchronize()

    sync_all()
    warmup_s = time.perf_counter() - t_warm
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss, _ = step()
    sync_all()
    elapsed = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss_val = float(loss)

    probe_out = os.environ.get("RTSEG_PROBE_OPS")
    if probe_out and rank == 0:  # one extra step: large non-kernel aten ops (tools/probe_step_ops.py)
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from tools.probe_step_ops import OpProbe

        probe = OpProbe()
        with probe:
            step()
        torch.cuda.synchronize()
        with open(probe_out, "w") as f:
            f.write(probe.report())

    if a.profile_steps > 0 and rank == 0:
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(a.profile_steps):
                step()
            torch.cuda.synchronize()
        os.makedirs("gpurun_out", exist_ok=True)
        with open("gpurun_out/torch_profile.txt", "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))

    ms = elapsed / a.steps * 1e3
    imgs_per_s = a.batch * world * a.steps / elapsed
    extra = {"loss_last": loss_val, "per_gpu_batch": a.batch,
             "peak_mem_gb": torch.cuda.max_memory_allocated(dev) / 2 ** 30,
             "hip_ext_loaded": bool(ops.load()), "channels_last": cfg.channels_last,
             "fused_loss": cfg.fused_loss, "miopen_find_mode": bool(cfg.cudnn_benchmark),
             "warmup_s": round(warmup_s, 1),
             # the optimizer step (+ parameter EMA) ran as the single fused HIP launch
             "fused_optimizer_step": bool(getattr(trainer.optimizer, "last_step_fused", False))}
    from realtime_semantic_segmentation_pytorch_amd.ops.conv import decisions

    picks = {}
    for k, (_, name, _t) in decisions().items():
        tag = f"{k[0]}:{name}"
        picks[tag] = picks.get(tag, 0) + 1
    extra["conv_kernel_choices"] = dict(sorted(picks.items()))  # per layer shape, per pass
    dec_out = os.environ.get("RTSEG_DECISIONS_OUT")
    if dec_out and rank == 0:  # full per-shape table: key -> (choice, [ms per candidate])
        with open(dec_out, "w") as f:
            for k, (_, name, ts) in sorted(decisions().items(), key=lambda kv: str(kv[0])):
                f.write(f"{k}\t{name}\t{ts}\n")
    if rank == 0 and not a.no_infer:
        m = de_parallel(trainer.model)
        tag = f"{a.height}x{a.width}"
        extra[f"infer_fps_bf16_bs1_{tag}"] = round(infer_fps(m, a.height, a.width, torch.bfloat16,
                                                             cfg.channels_last), 2)
        extra[f"infer_fps_fp32_bs1_{tag}"] = round(infer_fps(m, a.height, a.width, torch.float32,
                                                             cfg.channels_last), 2)
        if a.model == "ddrnet":
            # the README's own FPS row: DDRNet-23-slim, 1024x512, fp32, batch 1 (use_aux as in MyConfig)
            from realtime_semantic_segmentation_pytorch_amd.models import get_model

            sc = make_config(a, world)
            sc.arch_type = "DDRNet-23-slim"
            slim = get_model(sc).to(dev)
            fps = infer_fps(slim, a.height // 2, a.width // 2, torch.float32, cfg.channels_last)
            extra["ddrnet23slim_fps_fp32_bs1_512x1024"] = round(fps, 2)
            extra["ddrnet23slim_fps_vs_readme_rtx2080"] = round(fps / README_FPS_DDRNET23_SLIM, 3)
    if dist.is_initialized():
        barrier()
    if rank == 0:
        out = {
            "metric": "train_images_per_sec",
            "value": round(imgs_per_s, 3),
            "unit": "images/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if a.fp32 else "bf16",
            "data": f"synthetic (device-resident random {a.height}x{a.width} images, blocky 19-class masks, "
                    "random-init weights)",
            "config": {"model": a.arch if a.model == "ddrnet" else f"{a.model}-{a.arch}" if a.model in (
                           "stdc", "ppliteseg") else a.model,
                       "global_batch": a.batch * world,
                       "seq_len": f"{a.height}x{a.width}", "parallelism": f"dp{world}",
                       "num_class": 19, "loss": ("ohem+detail" if a.detail_head else "ohem+aux" if cfg.use_aux else "ohem")
                       + ("+kd(deeplabv3p-r101)" if a.kd else ""),
                       "optimizer": "sgd+onecycle+ema"},
            "extra": extra,
        }
        print(json.dumps(out), flush=True)
    hb.set()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
