"""Numerics bisection of one training step (BASELINE configs 2-4) against an fp64 reference.

For each model the step's loss and per-parameter gradients are computed

* in fp64 on the CPU (stock PyTorch, NCHW): the yardstick -- exact up to fp64 rounding, so it
  also judges the stock fp32 GPU path (whose channels-last MIOpen convs are not exact);
* on the GPU: stock fp32, stock bf16 (twice: the run-to-run spread), the HIP fp32 and bf16
  paths, and the HIP paths with ONE kernel family at a time sent back to its stock formulation
  (``RTSEG_HIP_OFF=<family>``; convs: ``RTSEG_CONV_MFMA=0``).

A family whose removal moves the HIP path's cosine distribution onto stock's is the one that
opens the gap.  Prints one summary row per variant and the worst parameters side by side.
Reference training step: core/seg_trainer.py:38-119; detail head :68-82.

    python tools/probe_numerics_bisect.py --models bisenetv2_aux,stdc2_detail [--size 256x512]
"""
import argparse
import copy
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.datasets import DeviceBatches  # noqa: E402

MODELS = {
    "ddrnet23_aux": dict(model="ddrnet", arch_type="DDRNet-23", use_aux=True),
    "bisenetv2_aux": dict(model="bisenetv2", arch_type=None, use_aux=True),
    "stdc2_detail": dict(model="stdc", arch_type=None, encoder_type="stdc2", use_aux=False, use_detail_head=True),
    "stdc2_aux": dict(model="stdc", arch_type=None, encoder_type="stdc2", use_aux=True),
}
FAMILIES = ["bn", "dw", "pool", "interp", "loss", "detail", "gate", "act", "deconv", "shuffle"]
ENV_KEYS = ("RTSEG_DISABLE_HIP", "RTSEG_CONV_MFMA", "RTSEG_HIP_OFF")


def variants(families, fp32_bisect):
    v = [("stock_fp32", False, {"RTSEG_DISABLE_HIP": "1"}),
         ("stock_bf16", True, {"RTSEG_DISABLE_HIP": "1"}),
         ("stock_bf16_rerun", True, {"RTSEG_DISABLE_HIP": "1"}),
         ("hip_fp32", False, {}),
         ("hip_bf16", True, {"RTSEG_CONV_MFMA": "1"}),
         ("hip_bf16_auto", True, {}),
         ("hip_bf16-conv", True, {"RTSEG_CONV_MFMA": "0"})]
    v += [(f"hip_bf16-{f}", True, {"RTSEG_CONV_MFMA": "1", "RTSEG_HIP_OFF": f}) for f in families]
    if fp32_bisect:
        v += [(f"hip_fp32-{f}", False, {"RTSEG_HIP_OFF": f}) for f in families]
    return v


def make_trainer(kw, size, bs):
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE") + ENV_KEYS:
        os.environ.pop(k, None)
    c = BaseConfig()
    c.dataset, c.num_class = "cityscapes", 19
    for k, v in kw.items():
        setattr(c, k, v)
    c.synthetic_data, c.synthetic_len, c.synthetic_size = True, 8, size
    c.crop_size, c.crop_h, c.crop_w = size[0], size[0], size[1]
    c.train_bs, c.val_bs, c.total_epoch = bs, bs, 2
    c.amp_training, c.amp_dtype, c.channels_last = True, "bf16", True
    c.base_workers, c.use_tb, c.save_ckpt, c.load_ckpt, c.use_ema = 0, False, False, False, False
    c.save_dir = "/tmp/probe_bisect"
    c.init_dependent_config()
    tr = SegTrainer(c)
    tr.model.train()
    return tr


def step(tr, imgs, masks, amp):
    tr.config.amp_training = amp
    tr.model.zero_grad(set_to_none=True)
    loss, _, extras = tr.compute_loss(imgs, masks)
    loss.backward()
    g = {n: p.grad.detach().double().cpu() for n, p in tr.model.named_parameters() if p.grad is not None}
    ex = {k: float(v.detach()) for k, v in extras.items() if isinstance(v, torch.Tensor) and v.numel() == 1}
    return float(loss.detach()), g, ex


def reference_fp64(tr, imgs, masks):
    """The same step in fp64 on the CPU (NCHW, every op on its stock PyTorch formulation)."""
    model_gpu = tr.model
    m64 = copy.deepcopy(model_gpu).cpu().double().to(memory_format=torch.contiguous_format)
    m64.train()
    tr.model = m64
    try:
        x = imgs.detach().cpu().double().contiguous()
        loss, g, ex = step(tr, x, masks.cpu(), amp=False)
    finally:
        tr.model = model_gpu
    return loss, g, ex


def cosines(g, ref):
    out = {}
    for n, r in ref.items():
        if n not in g or r.norm() <= 1e-12:
            continue
        a = g[n].flatten()
        b = r.flatten()
        out[n] = float(torch.dot(a, b) / (a.norm() * b.norm()).clamp_min(1e-300))
    return out


def summarize(c):
    v = sorted(c.values())
    n = len(v)
    return dict(n=n, median=v[n // 2], p10=v[n // 10], min=v[0], below09=sum(x < 0.9 for x in v),
                below099=sum(x < 0.99 for x in v))


def run_model(name, size, bs, families, fp32_bisect, worst):
    tr = make_trainer(MODELS[name], size, bs)
    imgs, masks = DeviceBatches(bs, size, 19, 255, device=tr.device, pool=1, channels_last=True, seed=0).next()
    t0 = time.time()
    loss64, g64, ex64 = reference_fp64(tr, imgs, masks)
    print(f"[{name}] fp64 CPU reference: loss {loss64:.6f} {ex64} ({time.time() - t0:.1f} s)", flush=True)
    res = {}
    for vname, amp, env in variants(families, fp32_bisect):
        for k in ENV_KEYS:
            os.environ.pop(k, None)
        os.environ.update(env)
        try:
            res[vname] = step(tr, imgs, masks, amp)
        except Exception as e:  # noqa: BLE001 - a family whose stock formulation rejects the input
            print(f"[{name}] {vname}: FAILED {type(e).__name__}: {e}", flush=True)
    for k in ENV_KEYS:
        os.environ.pop(k, None)
    rows = {}
    cos64 = {v: cosines(r[1], g64) for v, r in res.items()}
    cos32 = {v: cosines(r[1], res["stock_fp32"][1]) for v, r in res.items() if v != "stock_fp32"}
    print(f"[{name}] {'variant':<22}{'loss':>12}{'rel.err':>10}{'med64':>9}{'p10_64':>9}{'min64':>9}"
          f"{'<.9':>5}{'<.99':>5}{'med32':>9}{'p10_32':>9}  extras", flush=True)
    for v, (loss, g, ex) in res.items():
        s = summarize(cos64[v])
        s32 = summarize(cos32[v]) if v in cos32 else None
        rows[v] = dict(loss=loss, rel_err=(loss - loss64) / abs(loss64), extras=ex, vs_fp64=s, vs_fp32=s32)
        print(f"[{name}] {v:<22}{loss:12.6f}{rows[v]['rel_err']:10.5f}{s['median']:9.5f}{s['p10']:9.5f}"
              f"{s['min']:9.5f}{s['below09']:5d}{s['below099']:5d}"
              + (f"{s32['median']:9.5f}{s32['p10']:9.5f}" if s32 else " " * 18) + f"  {ex}", flush=True)
    # the worst parameters of the HIP paths, side by side with stock
    cols = [v for v in ("stock_fp32", "stock_bf16", "stock_bf16_rerun", "hip_fp32", "hip_bf16") if v in cos64]
    order = sorted(cos64["hip_bf16"], key=lambda n: cos64["hip_bf16"][n])[:worst]
    order += [n for n in sorted(cos64["hip_fp32"], key=lambda n: cos64["hip_fp32"][n])[:worst] if n not in order]
    print(f"[{name}] worst parameters (cosine to fp64; |g| = fp64 gradient norm)")
    print(f"[{name}] {'param':<56}{'|g|':>10}" + "".join(f"{c[:14]:>15}" for c in cols))
    for n in order:
        print(f"[{name}] {n:<56}{float(g64[n].norm()):10.2e}" + "".join(f"{cos64[c].get(n, float('nan')):15.5f}"
                                                                     for c in cols))
    return dict(loss_fp64=loss64, extras_fp64=ex64, variants=rows,
                worst={n: {c: cos64[c].get(n) for c in cols} for n in order})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="ddrnet23_aux,bisenetv2_aux,stdc2_detail")
    ap.add_argument("--size", default="256x512")
    ap.add_argument("--bs", type=int, default=4)
    ap.add_argument("--families", default=",".join(FAMILIES))
    ap.add_argument("--fp32-bisect", action="store_true")
    ap.add_argument("--worst", type=int, default=12)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    size = tuple(int(v) for v in a.size.split("x"))
    fams = [f for f in a.families.split(",") if f]
    out = {}
    for m in a.models.split(","):
        out[m] = run_model(m, size, a.bs, fams, a.fp32_bisect, a.worst)
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
