"""End-to-end SegTrainer on CPU with synthetic Cityscapes-shaped data (plumbing config)."""
import os

import torch

from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer


def make_cfg(tmp_path, **kw):
    c = BaseConfig()
    c.dataset = "cityscapes"
    c.num_class = 19
    c.model = "ddrnet"
    c.use_aux = True
    c.synthetic_data = True
    c.synthetic_len = 4
    c.synthetic_size = (64, 128)
    c.crop_size = 64
    c.train_bs = 2
    c.val_bs = 2
    c.total_epoch = 2
    c.base_workers = 0
    c.save_dir = str(tmp_path / "save")
    c.use_tb = True
    c.device = "cpu"
    c.use_ema = True
    for k, v in kw.items():
        setattr(c, k, v)
    c.init_dependent_config()
    return c


def test_train_validate_checkpoint_resume(tmp_path, monkeypatch):
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    cfg = make_cfg(tmp_path)
    tr = SegTrainer(cfg)
    tr.run(cfg)
    last = os.path.join(cfg.save_dir, "last.pth")
    best = os.path.join(cfg.save_dir, "best.pth")
    assert os.path.isfile(last) and os.path.isfile(best)
    ck = torch.load(last, weights_only=True)
    assert set(["cur_epoch", "best_score", "state_dict", "optimizer", "scheduler"]) <= set(ck)
    assert ck["cur_epoch"] == 1
    bk = torch.load(best, weights_only=True)
    assert bk["optimizer"] is None and bk["scheduler"] is None
    assert os.path.isfile(os.path.join(cfg.save_dir, "tb_logs", "scalars.jsonl"))



def test_resume_after_interruption(tmp_path, monkeypatch):
    """Kill after epoch 0 (only last.pth written), restart, continue at epoch 1."""
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    cfg = make_cfg(tmp_path, total_epoch=3)
    tr = SegTrainer(cfg)
    tr.parallel_model(cfg)
    tr.cur_epoch = 0
    tr.train_one_epoch(cfg)
    tr.save_ckpt(cfg)
    ema_ref = {k: v.clone() for k, v in tr.ema_model.ema.state_dict().items()}
    sched_ref = tr.scheduler.last_epoch
    del tr
    cfg2 = make_cfg(tmp_path, total_epoch=3)
    tr2 = SegTrainer(cfg2)
    assert tr2.cur_epoch == 1
    assert tr2.train_itrs == cfg2.iters_per_epoch
    assert tr2.scheduler.last_epoch == sched_ref
    for k, v in tr2.ema_model.ema.state_dict().items():
        torch.testing.assert_close(v, ema_ref[k])
    tr2.run(cfg2)
    assert torch.load(os.path.join(cfg2.save_dir, "last.pth"), weights_only=True)["cur_epoch"] == 2


def test_train_step_reduces_loss_cpu(tmp_path, monkeypatch):
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    cfg = make_cfg(tmp_path, model="ddrnet", use_aux=True, total_epoch=50, optimizer_type="adam")
    tr = SegTrainer(cfg)
    tr.model.train()
    imgs, masks = next(iter(tr.train_loader))
    losses = [float(tr.train_step(imgs, masks)[0]) for _ in range(12)]
    assert losses[-1] < losses[0]
