"""End-to-end learning on a LEARNABLE synthetic task (labels = colour-coded blocks of the image,
``config.synthetic_learnable``): ``run`` trains, validates the EMA model every epoch, keeps the
best mIoU in ``best.pth`` (EMA weights) and ``val_best`` re-validates that checkpoint.

The reference's only correctness evidence is Cityscapes val mIoU (README.md:133-203); there is no
dataset here, so this checks the same machinery -- train -> validate(EMA) -> best.pth -> val_best
(core/seg_trainer.py:123-152, core/base_trainer.py:71-109, 165-186) -- on a task whose mIoU must
rise when training works.
"""
import os

import pytest
import torch

from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer


def _cfg(tmp_path, device, **kw):
    c = BaseConfig()
    c.dataset, c.num_class = "cityscapes", 19
    c.synthetic_data, c.synthetic_learnable = True, True
    c.base_workers, c.use_tb, c.save_ckpt, c.use_ema = 0, False, True, True
    c.save_dir = str(tmp_path / "save")
    c.load_ckpt = False
    c.device = device
    c.begin_val_epoch, c.val_interval = 0, 1
    for k, v in kw.items():
        setattr(c, k, v)
    c.init_dependent_config()
    return c


def _train(cfg):
    tr = SegTrainer(cfg)
    history = []
    validate = tr.validate

    def recording_validate(config, val_best=False):
        score = validate(config, val_best)
        history.append((val_best, score))
        return score

    tr.validate = recording_validate
    tr.run(cfg)
    return tr, history


def _check(tr, history, cfg, floor):
    epochs = [s for vb, s in history if not vb]
    finals = [s for vb, s in history if vb]
    assert len(epochs) == cfg.total_epoch and len(finals) == 1, history
    assert os.path.isfile(os.path.join(cfg.save_dir, "best.pth"))
    best = max(epochs)
    assert tr.best_score == pytest.approx(best)
    # the learnable task is learnt: validation mIoU climbs well above the first epoch's ...
    assert best >= floor and best > epochs[0], epochs
    # ... and val_best re-validates best.pth (the EMA weights of the best epoch) to the same score
    assert finals[0] == pytest.approx(best, abs=2e-3), (finals, best)


def test_learnable_task_converges_cpu(tmp_path, monkeypatch):
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    cfg = _cfg(tmp_path, "cpu", model="fastscnn", synthetic_len=64, synthetic_size=(64, 128), crop_size=64,
               synthetic_cell=32, train_bs=8, val_bs=8, total_epoch=16, optimizer_type="adam",
               lr_policy="linear", amp_training=False)
    tr, history = _train(cfg)
    _check(tr, history, cfg, floor=0.5)


@pytest.mark.gpu
@pytest.mark.parametrize("model,arch", [("ddrnet", "DDRNet-23-slim"), ("bisenetv2", None)])
def test_learnable_task_converges_gpu(tmp_path, monkeypatch, model, arch):
    """bf16, channels-last, every HIP kernel, the fused optimizer + EMA: val mIoU > 0.9."""
    from realtime_semantic_segmentation_pytorch_amd import ops

    assert ops.load()
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "RTSEG_DISABLE_HIP"):
        monkeypatch.delenv(k, raising=False)
    cfg = _cfg(tmp_path, "cuda", model=model, arch_type=arch, use_aux=model == "bisenetv2",
               synthetic_len=96, synthetic_size=(256, 512), crop_size=256, synthetic_cell=64, train_bs=8,
               val_bs=8, total_epoch=10, optimizer_type="adam", lr_policy="linear", amp_training=True,
               amp_dtype="bf16", channels_last=True)
    tr, history = _train(cfg)
    assert tr.ema_fused
    _check(tr, history, cfg, floor=0.9)
