"""Model-level numerics of the bench configuration on the GPU.

* one DDRNet-23 (+aux) training step in bf16 / channels-last with every HIP kernel on (MFMA
  conv fwd/dgrad/wgrad, fused BN, fused OHEM, interp) vs the same step with
  ``RTSEG_DISABLE_HIP=1`` (stock PyTorch / MIOpen): loss and gradient agreement;
* 200 steps overfitting one synthetic batch with every HIP kernel on: the loss must fall;
* an fp16 + GradScaler step (``amp_dtype='fp16'``, reference core/base_trainer.py:30).
Reference training step: core/seg_trainer.py:38-119.
"""
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


def _grads(tr, imgs, masks):
    tr.model.zero_grad(set_to_none=True)
    loss, _, _ = tr.compute_loss(imgs, masks)
    loss.backward()
    g = {n: p.grad.detach().float().clone() for n, p in tr.model.named_parameters() if p.grad is not None}
    return float(loss), g


def test_ddrnet23_bf16_step_hip_vs_stock(tmp_path, monkeypatch):
    tr = _trainer(tmp_path)
    imgs, masks = _batch(tr)
    monkeypatch.setenv("RTSEG_CONV_MFMA", "1")  # our conv kernels on every eligible layer
    loss_hip, g_hip = _grads(tr, imgs, masks)
    monkeypatch.setenv("RTSEG_DISABLE_HIP", "1")
    loss_ref, g_ref = _grads(tr, imgs, masks)
    assert set(g_hip) == set(g_ref)
    assert abs(loss_hip - loss_ref) <= 2e-2 * abs(loss_ref), (loss_hip, loss_ref)
    n_hip = torch.sqrt(sum((g * g).sum() for g in g_hip.values()))
    n_ref = torch.sqrt(sum((g * g).sum() for g in g_ref.values()))
    assert abs(float(n_hip) - float(n_ref)) <= 5e-2 * float(n_ref), (float(n_hip), float(n_ref))
    # per-tensor direction: bf16 rounding and OHEM ties may move a few values, never a whole layer
    cos = {n: float(torch.nn.functional.cosine_similarity(g_hip[n].flatten(), g_ref[n].flatten(), dim=0))
           for n in g_ref if g_ref[n].norm() > 1e-6}
    bad = {n: c for n, c in cos.items() if c < 0.95}
    assert len(bad) <= len(cos) // 50, bad
    assert sorted(cos.values())[len(cos) // 2] > 0.99  # median layer


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
