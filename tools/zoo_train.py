"""Training throughput of every zoo model on one MI355X (synthetic 1024x2048 19-class data,
random init, bf16 autocast, channels-last, OHEM (+ aux heads where the model has them), fused
SGD + OneCycle + EMA): the same SegTrainer.train_step the trainer and bench.py run.

  python tools/zoo_train.py [--batch 8] [--steps 5] [--warmup 3] [--models a,b] [--out f.jsonl]

One JSON line per model (images/s, ms/step, peak memory); a model that fails is recorded with
its error and the sweep continues.  MIOpen find mode follows utils/runtime.py (verified models only).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.datasets import DeviceBatches  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.models import AUX_MODELS, MODEL_HUB  # noqa: E402


def config(key, a):
    c = BaseConfig()
    c.dataset, c.num_class, c.model = "cityscapes", 19, key
    c.use_aux = key in AUX_MODELS
    c.loss_type, c.optimizer_type = "ohem", "sgd"
    c.train_bs = a.batch
    c.synthetic_data, c.synthetic_len = True, a.batch
    c.crop_h, c.crop_w = a.height, a.width
    c.base_workers, c.save_ckpt, c.use_tb, c.load_ckpt = 0, False, False, False
    c.save_dir = "/tmp/rtseg_zoo_train"
    c.use_ema, c.is_testing = True, False
    # bf16 autocast like bench.py (BaseConfig's default is fp32, on which the MFMA conv kernels
    # do not run: round 2's sweep measured fp32 by mistake); --fp32 for that column
    c.amp_training, c.amp_dtype = not a.fp32, "bf16"
    # --graph-step: forward + loss + backward replayed from one captured HIP graph after the
    # warm-up (SegTrainer.graph_step) -- the launch-bound small models (FDDWNet: 66 ms of kernels
    # in a 139 ms eager step, profiles/r4_zoo_models)
    c.graph_step = bool(a.graph_step)
    c.init_dependent_config()
    return c


def run(key, a):
    cfg = config(key, a)
    tr = SegTrainer(cfg)
    tr.model.train()
    data = DeviceBatches(a.batch, (a.height, a.width), cfg.num_class, cfg.ignore_index, device=tr.device,
                         pool=2, channels_last=cfg.channels_last, seed=7)
    torch.cuda.reset_peak_memory_stats()
    for i in range(a.warmup):
        t = time.perf_counter()
        tr.train_step(*data.next())
        torch.cuda.synchronize()
        print(f"[zoo_train] {key} warm-up step {i}: {time.perf_counter() - t:.2f} s", flush=True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss, _ = tr.train_step(*data.next())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    return {"model": key, "graph_step": bool(a.graph_step), "images_per_s": round(a.batch / dt, 2),
            "ms_per_step": round(dt * 1e3, 2),
            "loss": round(float(loss), 4), "aux": cfg.use_aux, "dtype": "fp32" if a.fp32 else "bf16",
            "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--width", type=int, default=2048)
    ap.add_argument("--models", default="")
    ap.add_argument("--fp32", action="store_true", help="no autocast (fp32 training)")
    ap.add_argument("--graph-step", action="store_true", help="replay the step from a captured HIP graph")
    ap.add_argument("--out", default="gpurun_out/zoo_train.jsonl")
    a = ap.parse_args()
    assert torch.cuda.is_available() and ops.load()
    import threading

    main_id = threading.get_ident()

    def beat():  # keeps a long autotune visible to the runner, with where the main thread is
        while True:
            time.sleep(60)
            fr, where = sys._current_frames().get(main_id), []
            while fr is not None and len(where) < 6:
                where.append(f"{os.path.basename(fr.f_code.co_filename)}:{fr.f_lineno}:{fr.f_code.co_name}")
                fr = fr.f_back
            print("[zoo_train] alive: " + " <- ".join(where), flush=True)

    threading.Thread(target=beat, daemon=True).start()
    keys = [k for k in a.models.split(",") if k] or sorted(MODEL_HUB)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "a") as f:
        for key in keys:
            t = time.perf_counter()
            try:
                rec = run(key, a)
            except Exception as e:  # noqa: BLE001 - record and continue with the next model
                rec = {"model": key, "error": f"{type(e).__name__}: {str(e)[:300]}"}
                if "illegal memory access" in str(e) or "hipError" in str(e):
                    print(json.dumps(rec), flush=True)
                    f.write(json.dumps(rec) + "\n")
                    raise  # the device is unusable after a fault: stop here
            rec["wall_s"] = round(time.perf_counter() - t, 1)
            print(json.dumps(rec), flush=True)
            f.write(json.dumps(rec) + "\n")
            f.flush()
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
