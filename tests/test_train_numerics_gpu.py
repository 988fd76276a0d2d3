"""Model-level numerics of the bench configuration on the GPU.

* one training step of BASELINE configs 2-4 (DDRNet-23 + aux, BiSeNetV2 + aux, STDC2 + detail)
  in bf16 / channels-last with every HIP kernel on (MFMA conv fwd/dgrad/wgrad, fused BN, fused
  OHEM, interp, ...), in HIP fp32 and in stock bf16 (``RTSEG_DISABLE_HIP=1``), all against the
  same step in fp64 on the CPU (tools/probe_numerics_bisect.py prints the per-family bisection
  and the per-parameter table);
* 200 steps overfitting one synthetic batch with every HIP kernel on: the loss must fall;
* an fp16 + GradScaler step (``amp_dtype='fp16'``, reference core/base_trainer.py:30).
Reference training step: core/seg_trainer.py:38-119.
"""
import copy
import os

import pytest
import torch

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _env(monkeypatch):
    assert ops.load(), "HIP extension must load on the GPU box"
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "RTSEG_DISABLE_HIP"):
        monkeypatch.delenv(k, raising=False)


def _trainer(tmp_path, **kw):
    from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer

    c = BaseConfig()
    c.dataset, c.num_class, c.model, c.arch_type, c.use_aux = "cityscapes", 19, "ddrnet", "DDRNet-23", True
    c.synthetic_data, c.synthetic_len, c.synthetic_size = True, 8, (256, 512)
    c.crop_size, c.crop_h, c.crop_w = 256, 256, 512
    c.train_bs, c.val_bs, c.total_epoch = 4, 4, 200
    c.amp_training, c.amp_dtype, c.channels_last = True, "bf16", True
    c.base_workers, c.use_tb, c.save_ckpt, c.load_ckpt, c.use_ema = 0, False, False, False, True
    c.save_dir = str(tmp_path / "save")
    for k, v in kw.items():
        setattr(c, k, v)
    c.init_dependent_config()
    tr = SegTrainer(c)
    tr.model.train()
    return tr


def _batch(tr, seed=0):
    from realtime_semantic_segmentation_pytorch_amd.datasets import DeviceBatches

    data = DeviceBatches(4, (256, 512), 19, 255, device=tr.device, pool=1, channels_last=True, seed=seed)
    return data.next()


def _grads(tr, imgs, masks, amp=True):
    tr.config.amp_training = amp
    tr.model.zero_grad(set_to_none=True)
    loss, _, _ = tr.compute_loss(imgs, masks)
    loss.backward()
    g = {n: p.grad.detach().double().cpu() for n, p in tr.model.named_parameters() if p.grad is not None}
    return float(loss.detach()), g


def _grads_fp64_cpu(tr, imgs, masks):
    """The same step in fp64 on the CPU (NCHW, stock PyTorch formulation of every op): the
    yardstick.  The stock fp32 GPU step is NOT exact -- PyTorch's channels-last avg_pool2d
    backward misplaces the gradient of padded windows on this ROCm build (README, ``pool.hip``),
    which alone puts 12 of BiSeNetV2's gradients below cosine 0.9 (profiles/r4_numerics)."""
    model = tr.model
    tr.model = copy.deepcopy(model).cpu().double().to(memory_format=torch.contiguous_format)
    try:
        return _grads(tr, imgs.detach().cpu().double().contiguous(), masks.cpu(), amp=False)
    finally:
        tr.model = model


def _cos(g, ref, live):
    return {n: float(torch.dot(g[n].flatten(), ref[n].flatten()) / (g[n].norm() * ref[n].norm()))
            for n in live}


# BASELINE configs 2-4: DDRNet-23 + aux, BiSeNetV2 + 4 aux heads, STDC2 + detail head (OHEM).
# Measured on MI355X against the fp64 CPU step (profiles/r4_numerics/bisect.txt), median cosine /
# parameters < 0.9: DDRNet-23 stock bf16 0.828 / 124, HIP bf16 0.838 / 122; BiSeNetV2 0.896 / 86 vs
# 0.926 / 52; STDC2 + detail 0.394 / 151 vs 0.414 / 147 (random-init BN chains amplify bf16
# rounding; two stock bf16 runs already differ).  HIP fp32: median 0.99998+, p10 0.9999 on all three.
_STEP_MODELS = {
    "ddrnet23_aux": {},
    "bisenetv2_aux": {"model": "bisenetv2", "arch_type": None},
    "stdc2_detail": {"model": "stdc", "arch_type": None, "encoder_type": "stdc2", "use_aux": False,
                     "use_detail_head": True},
}


@pytest.mark.parametrize("name", sorted(_STEP_MODELS))
def test_bf16_step_vs_fp64_reference(tmp_path, monkeypatch, name):
    """One training step's loss and gradients against the fp64 CPU step.

    * HIP fp32 (our BN / loss / pooling / interp / depth-wise kernels around MIOpen convs) is
      exact to fp32: loss within 1e-5, gradient cosine median > 0.9999 and p10 > 0.999;
    * HIP bf16 (MFMA convs, fused BN, residual-gradient hand-off, OHEM / detail loss, ...) is at
      least as close as stock PyTorch bf16 on the same step: median cosine >= stock's - 5e-3, no
      more parameters below 0.9 than stock (+2 %), loss within 2 % of fp64.
    Parameters whose fp64 gradient is numerically zero (norm < 1e-4 x the median norm: BN weights
    of GatherExpansion branches whose output feeds a scale-invariant BN) are not judged -- their
    cosine is rounding noise on any path.  The stock bf16 loss is reported, not judged: on STDC2 it
    is 2.3 % off fp64 because the reference formulation thresholds the detail target computed in
    bf16 under autocast (core/seg_trainer.py:72-76); ours computes it exactly (0.27 %)."""
    tr = _trainer(tmp_path, **_STEP_MODELS[name])
    imgs, masks = _batch(tr)
    loss_64, g_64 = _grads_fp64_cpu(tr, imgs, masks)
    monkeypatch.setenv("RTSEG_DISABLE_HIP", "1")
    loss_sb, g_sb = _grads(tr, imgs, masks)
    monkeypatch.delenv("RTSEG_DISABLE_HIP")
    monkeypatch.setenv("RTSEG_CONV_MFMA", "1")  # our conv kernels on every eligible layer
    loss_hb, g_hb = _grads(tr, imgs, masks)
    monkeypatch.delenv("RTSEG_CONV_MFMA")
    loss_hf, g_hf = _grads(tr, imgs, masks, amp=False)
    assert set(g_hb) == set(g_64) == set(g_hf) == set(g_sb)
    norms = sorted(float(g.norm()) for g in g_64.values())
    live = [n for n, g in g_64.items() if float(g.norm()) > 1e-4 * norms[len(norms) // 2]]
    # BiSeNetV2: 157 of 189 (conv biases ahead of a BN and BN weights ahead of a scale-invariant BN
    # have mathematically zero gradients)
    assert len(live) >= 0.75 * len(g_64), (len(live), len(g_64))
    c_sb, c_hb, c_hf = (sorted(_cos(g, g_64, live).values()) for g in (g_sb, g_hb, g_hf))
    med, p10 = len(live) // 2, len(live) // 10
    rel = {k: (v - loss_64) / abs(loss_64) for k, v in (("stock_bf16", loss_sb), ("hip_bf16", loss_hb),
                                                       ("hip_fp32", loss_hf))}
    print(f"{name}: loss rel. error vs fp64 {rel}; cos median stock-bf16 {c_sb[med]:.4f} hip-bf16 {c_hb[med]:.4f} "
          f"hip-fp32 {c_hf[med]:.6f}; p10 hip-fp32 {c_hf[p10]:.6f}; <0.9: stock {sum(c < 0.9 for c in c_sb)} "
          f"hip {sum(c < 0.9 for c in c_hb)} of {len(live)}")
    assert abs(rel["hip_fp32"]) <= 1e-5, rel
    assert c_hf[med] > 0.9999 and c_hf[p10] > 0.999, (c_hf[med], c_hf[p10])
    assert abs(rel["hip_bf16"]) <= 2e-2, rel
    assert c_hb[med] >= c_sb[med] - 5e-3, (c_hb[med], c_sb[med])
    assert sum(c < 0.9 for c in c_hb) <= sum(c < 0.9 for c in c_sb) + max(1, int(0.02 * len(live)))


def test_ddrnet23_overfits_one_batch_with_hip_kernels(tmp_path):
    tr = _trainer(tmp_path, optimizer_type="adam", lr_policy="linear")
    imgs, masks = _batch(tr, seed=3)
    losses = []
    for _ in range(200):
        loss, _ = tr.train_step(imgs, masks)
        losses.append(float(loss))
    assert all(torch.isfinite(torch.tensor(losses)))
    first, last = sum(losses[:5]) / 5, sum(losses[-5:]) / 5
    assert last <= 0.5 * first, (first, last)


def test_fp16_gradscaler_step(tmp_path):
    tr = _trainer(tmp_path, amp_dtype="fp16", model="bisenetv2", arch_type=None)
    assert tr.scaler.is_enabled() and not tr.ema_fused
    imgs, masks = _batch(tr, seed=5)
    before = {n: p.detach().clone() for n, p in tr.model.named_parameters()}
    for _ in range(3):
        loss, _ = tr.train_step(imgs, masks)
        assert torch.isfinite(loss)
    assert tr.scaler.get_scale() > 0
    moved = sum(int(not torch.equal(before[n], p.detach())) for n, p in tr.model.named_parameters())
    assert moved >= len(before) // 2
