"""User-facing surfaces on CPU: CLI strictness, augmentation randomness per epoch, the labelme
converter -> Custom dataset round trip, predict end to end, and the step / linear / OneCycle
LR policies (reference: configs/parser.py, datasets/cityscapes.py:115-124,
utils/check_datasets.py:14-112, datasets/custom.py:12-84, core/seg_trainer.py:154-191,
utils/scheduler.py:5-25)."""
import base64
import io
import json
import os

import numpy as np
import pytest
import torch
from PIL import Image

from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig, MyConfig, load_parser
from realtime_semantic_segmentation_pytorch_amd.datasets import Cityscapes, Custom, EpochSampler, get_loader


@pytest.fixture(autouse=True)
def _single_process(monkeypatch):
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)


# --------------------------------------------------------------------------------- CLI
def test_parser_rejects_unknown_flags():
    with pytest.raises(SystemExit):
        load_parser(MyConfig(), ["--modle", "ddrnet"])
    cfg = load_parser(MyConfig(), ["--model", "ddrnet", "--train_bs", "4"])
    assert cfg.model == "ddrnet" and cfg.train_bs == 4


# ------------------------------------------------------------------------ augmentation
def _fake_cityscapes(root, n=3, h=48, w=96):
    rng = np.random.default_rng(0)
    for i in range(n):
        for mode in ("train", "val"):
            d_img = os.path.join(root, "leftImg8bit", mode, "city")
            d_msk = os.path.join(root, "gtFine", mode, "city")
            os.makedirs(d_img, exist_ok=True)
            os.makedirs(d_msk, exist_ok=True)
            Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8)).save(
                os.path.join(d_img, f"city_{i:06d}_000019_leftImg8bit.png"))
            Image.fromarray(rng.integers(0, 34, (h, w), dtype=np.uint8)).save(
                os.path.join(d_msk, f"city_{i:06d}_000019_gtFine_labelIds.png"))


def _aug_cfg(root, **kw):
    c = BaseConfig()
    c.dataset, c.num_class, c.data_root = "cityscapes", 19, str(root)
    c.crop_size, c.randscale = 32, [-0.5, 1.0]
    c.brightness = c.contrast = c.saturation = 0.5
    c.h_flip = 0.5
    c.train_bs = c.val_bs = 2
    c.DDP, c.gpu_num = False, 1
    for k, v in kw.items():
        setattr(c, k, v)
    c.init_dependent_config()
    return c


def test_augmentation_is_fresh_every_epoch_and_reproducible(tmp_path):
    _fake_cityscapes(tmp_path)
    cfg = _aug_cfg(tmp_path)
    ds = Cityscapes(cfg, "train")
    a0, m0 = ds[(1, 0)]
    a1, m1 = ds[(1, 1)]
    assert a0.shape == a1.shape == (3, 32, 32)
    assert not torch.equal(a0, a1), "same index must get a different augmentation in epoch 1"
    b0, n0 = Cityscapes(cfg, "train")[(1, 0)]  # a rerun with the same seed is bit-identical
    assert torch.equal(a0, b0) and torch.equal(m0, n0)
    c0, _ = Cityscapes(_aug_cfg(tmp_path, random_seed=7), "train")[(1, 0)]
    assert not torch.equal(a0, c0), "the seed must enter the stream"


@pytest.mark.parametrize("workers", [0, 2])
def test_loader_carries_epoch_to_workers(tmp_path, workers):
    _fake_cityscapes(tmp_path, n=4)
    cfg = _aug_cfg(tmp_path, num_workers=workers)
    train_loader, _ = get_loader(cfg)
    assert isinstance(train_loader.sampler, EpochSampler)
    epochs = []
    for epoch in (0, 1):
        train_loader.sampler.set_epoch(epoch)
        batches = [(x.clone(), y.clone()) for x, y in train_loader]
        assert len(batches) == 2
        for x, y in batches:
            assert x.shape == (2, 3, 32, 32) and y.dtype == torch.int64
            assert int(y.max()) <= 255 and int(y.min()) >= 0
        epochs.append(torch.cat([b[0] for b in batches]))
    assert not torch.equal(epochs[0], epochs[1])


def test_loader_streams_match_across_worker_counts(tmp_path):
    """The augmentation of a given (epoch, index) does not depend on the worker layout."""
    _fake_cityscapes(tmp_path, n=4)
    outs = []
    for workers in (0, 2):
        cfg = _aug_cfg(tmp_path, num_workers=workers)
        ds = Cityscapes(cfg, "train")
        outs.append(torch.stack([ds[(i, 3)][0] for i in range(4)]))
    assert torch.equal(outs[0], outs[1])


# --------------------------------------------------------------- labelme -> Custom
def _png_b64(arr):
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="PNG")
    return base64.b64encode(buf.getvalue()).decode()


def test_labelme_converter_and_custom_dataset(tmp_path):
    from realtime_semantic_segmentation_pytorch_amd.utils.check_datasets import check_semantic_segmentation_datasets

    lab = tmp_path / "labels"
    lab.mkdir()
    rng = np.random.default_rng(1)
    for i in range(20):
        img = rng.integers(0, 255, (40, 60, 3), dtype=np.uint8)
        shapes = [{"label": "car", "shape_type": "polygon", "points": [[5, 5], [30, 5], [30, 20], [5, 20]]},
                  {"label": "road" if i % 2 else "tree", "shape_type": "polygon",
                   "points": [[35, 25], [55, 25], [55, 38]]}]
        (lab / f"img{i:02d}.json").write_text(json.dumps({"imageData": _png_b64(img), "shapes": shapes,
                                                          "imagePath": f"img{i:02d}.png"}))
    names = check_semantic_segmentation_datasets(str(tmp_path))
    assert names["_background"] == 0 and set(names) == {"_background", "car", "road", "tree"}
    out = tmp_path / "out"
    tr = sorted(os.listdir(out / "train" / "imgs"))
    va = sorted(os.listdir(out / "val" / "imgs"))
    assert len(tr) == 19 and len(va) == 1  # 95 / 5 split
    m = np.asarray(Image.open(out / "train" / "masks" / tr[0]))
    assert m.shape == (40, 60) and m[10, 10] == names["car"] and m[0, 0] == 0
    cfg = BaseConfig()
    cfg.dataset, cfg.data_root, cfg.num_class = "custom", str(out), len(names)
    cfg.crop_size, cfg.train_size, cfg.test_size = 32, 48, 48
    cfg.init_dependent_config()
    ds = Custom(cfg, "train")
    assert ds.class_names == [k for k, _ in sorted(names.items(), key=lambda kv: kv[1])] and len(ds) == 19
    x, y = ds[(0, 0)]
    assert x.shape == (3, 32, 32) and 0.0 <= float(x.min()) and float(x.max()) <= 1.0
    assert int(y.max()) < len(names)
    xv, yv = Custom(cfg, "val")[0]
    assert xv.shape == (3, 48, 48) and yv.shape == (48, 48)


# ------------------------------------------------------------------------- predict
def test_predict_writes_masks_and_blends(tmp_path):
    from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer
    from realtime_semantic_segmentation_pytorch_amd.models import get_model

    folder = tmp_path / "imgs"
    folder.mkdir()
    rng = np.random.default_rng(2)
    for i in range(3):
        Image.fromarray(rng.integers(0, 255, (32, 64, 3), dtype=np.uint8)).save(folder / f"frame{i}.png")
    c = BaseConfig()
    c.dataset, c.num_class, c.model = "cityscapes", 19, "enet"
    c.is_testing, c.test_data_folder, c.test_bs = True, str(folder), 2
    c.save_dir = str(tmp_path / "save")
    c.blend_prediction, c.save_mask, c.blend_alpha = True, True, 0.3
    c.device = "cpu"
    c.base_workers = 0
    model = get_model(c)
    ck = tmp_path / "model.pth"
    torch.save({"state_dict": model.state_dict()}, ck)
    c.load_ckpt, c.load_ckpt_path = True, str(ck)
    c.init_dependent_config()
    c.load_ckpt_path = str(ck)
    tr = SegTrainer(c)
    tr.predict(c)
    out = tmp_path / "save" / "predicts"
    files = sorted(os.listdir(out))
    assert files == sorted([f"frame{i}.png" for i in range(3)] + [f"frame{i}_blend.png" for i in range(3)])
    mask = np.asarray(Image.open(out / "frame0.png"))
    assert mask.shape == (32, 64, 3)
    blend = np.asarray(Image.open(out / "frame0_blend.png"))
    raw = np.asarray(Image.open(folder / "frame0.png"))
    expect = np.asarray(Image.blend(Image.fromarray(raw), Image.fromarray(mask), 0.3))
    assert np.array_equal(blend, expect)


# ----------------------------------------------------------------------- schedulers
def _sched(policy, optimizer_type="sgd", **kw):
    from realtime_semantic_segmentation_pytorch_amd.utils.optim import get_scheduler

    c = BaseConfig()
    c.lr_policy, c.total_epoch, c.train_num, c.train_bs, c.DDP, c.gpu_num = policy, 10, 40, 4, False, 1
    c.warmup_epochs, c.step_size, c.lr = 2, 3, 0.1
    for k, v in kw.items():
        setattr(c, k, v)
    p = torch.nn.Parameter(torch.zeros(3))
    opt = (torch.optim.SGD([p], lr=c.lr, momentum=0.9) if optimizer_type == "sgd"
           else torch.optim.Adam([p], lr=c.lr))
    return c, opt, get_scheduler(c, opt)


def test_step_policy_decays_every_step_size_epochs():
    c, opt, s = _sched("step")
    assert c.iters_per_epoch == 10 and c.total_itrs == 100
    lrs = []
    for _ in range(c.total_itrs):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        s.step()
    assert lrs[0] == pytest.approx(0.1) and lrs[29] == pytest.approx(0.1)
    assert lrs[30] == pytest.approx(0.01) and lrs[60] == pytest.approx(1e-3) and lrs[99] == pytest.approx(1e-4)


def test_linear_policy_anneals_from_max_without_warmup():
    c, opt, s = _sched("linear")
    lrs = []
    for _ in range(c.total_itrs):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        s.step()
    assert lrs[0] == pytest.approx(0.1, rel=2e-2)  # pct_start = 0: no warm-up, starts at ~max_lr
    assert all(a >= b for a, b in zip(lrs, lrs[1:]))
    d = np.diff(np.asarray(lrs[1:]))
    assert np.allclose(d, d[0], rtol=1e-3, atol=1e-7)  # linear anneal: constant decrement
    assert lrs[-1] == pytest.approx(0.1 / 25 / 1e4, rel=5e-2, abs=1e-3)


@pytest.mark.parametrize("optimizer_type", ["sgd", "adam"])
def test_cos_warmup_cycles_momentum(optimizer_type):
    c, opt, s = _sched("cos_warmup", optimizer_type)
    key = "momentum" if optimizer_type == "sgd" else "betas"
    get = (lambda: opt.param_groups[0][key]) if optimizer_type == "sgd" else (lambda: opt.param_groups[0][key][0])
    lrs, moms = [], []
    for _ in range(c.total_itrs):
        lrs.append(opt.param_groups[0]["lr"])
        moms.append(get())
        opt.step()
        s.step()
    peak = int(np.argmax(lrs))
    assert lrs[0] == pytest.approx(0.1 / 25) and lrs[peak] == pytest.approx(0.1, rel=1e-3)
    assert peak == pytest.approx(0.2 * c.total_itrs, abs=2)  # warmup_epochs / total_epoch
    assert moms[0] == pytest.approx(0.95) and moms[peak] == pytest.approx(0.85, abs=1e-3)
    assert moms[-1] == pytest.approx(0.95, abs=1e-3)
    with pytest.raises(ValueError):  # stepping past total_itrs raises, as in the reference
        s.step()


def test_miopen_find_mode_only_on_verified_models(monkeypatch):
    """MIOpen's exhaustive solver search faulted the GPU on degenerate dilated convs (CFPNet at
    1024x512, LEDNet's dilation-17 (3,1) convs on a 16-row map at 128x256 once a trainer had
    switched find mode on for the whole pytest process): find mode is per model and the naive
    solvers -- the fallback for those geometries -- are only excluded by bench.py."""
    import torch

    from realtime_semantic_segmentation_pytorch_amd.utils.runtime import _NAIVE, configure_backend

    for k in _NAIVE:  # set-then-delete so monkeypatch restores the original state afterwards
        monkeypatch.setenv(k, "1")
        monkeypatch.delenv(k)
    saved = torch.backends.cudnn.benchmark
    try:
        configure_backend(True, model="ddrnet")
        assert torch.backends.cudnn.benchmark
        for key in ("lednet", "cfpnet", "enet", "smp"):
            configure_backend(True, model=key)
            assert not torch.backends.cudnn.benchmark, key
        assert all(k not in os.environ for k in _NAIVE)  # trainers keep the naive solvers
        configure_backend(True, model="ddrnet", exclude_naive=True)  # bench.py only
        assert all(os.environ[k] == "0" for k in _NAIVE)
    finally:
        torch.backends.cudnn.benchmark = saved
