"""Fused optimizer + EMA step on the production path (ops/optim.py, csrc/kernels/optim.hip).

* differential test: one DDRNet-23 channels-last model, the SAME gradients fed to
  ``FusedSGD`` / ``FusedAdam`` / ``FusedAdamW`` and to ``torch.optim``; every parameter and every
  state tensor is compared after each of several steps, and the fused kernel must have run;
* the weight gradients of channels-last convs arrive in the parameter's strides (no re-layout
  copy, no DDP bucket-stride mismatch, fused path eligible);
* the EMA model validated twice with training steps in between sees the new weights (the
  bf16 weight / BN coefficient caches fold in the raw-pointer write generation).
Reference: utils/optimizer.py:4-20, utils/model_ema.py:28-40."""
import copy

import pytest
import torch

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
from realtime_semantic_segmentation_pytorch_amd.models import get_model
from realtime_semantic_segmentation_pytorch_amd.ops.optim import FusedAdam, FusedAdamW, FusedSGD

pytestmark = pytest.mark.gpu


def _ddrnet(train=True):
    c = BaseConfig()
    c.model, c.arch_type, c.num_class, c.use_aux = "ddrnet", "DDRNet-23", 19, True
    torch.manual_seed(0)
    m = get_model(c).cuda().to(memory_format=torch.channels_last)
    return m.train(train)


def _real_grads(m):
    x = torch.randn(2, 3, 128, 256, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 19, (2, 128, 256), device="cuda")
    from realtime_semantic_segmentation_pytorch_amd.core.loss import SegCELoss

    loss_fn = SegCELoss()
    with torch.autocast("cuda", dtype=torch.bfloat16), ops.defer_final_upsample(True):
        out, (aux,) = m(x, is_training=True)
        loss = loss_fn(out, y) + loss_fn.aux(aux, y)
    loss.backward()
    return {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}


def test_channels_last_weight_grads_have_param_strides():
    m = _ddrnet()
    _real_grads(m)
    bad = [(n, tuple(p.stride()), tuple(p.grad.stride())) for n, p in m.named_parameters()
           if p.grad is not None and p.grad.stride() != p.stride()]
    assert not bad, bad[:5]


@pytest.mark.parametrize("kind", ["sgd", "adam", "adamw"])
def test_fused_step_matches_torch_per_tensor(kind):
    m = _ddrnet()
    grads = _real_grads(m)
    ref_m, fus_m = copy.deepcopy(m), copy.deepcopy(m)
    rp = [p for _, p in ref_m.named_parameters()]
    fp = [p for _, p in fus_m.named_parameters()]
    names = [n for n, _ in m.named_parameters()]
    if kind == "sgd":
        ref = torch.optim.SGD(rp, lr=0.05, momentum=0.9, weight_decay=1e-4, foreach=True)
        fus = FusedSGD(fp, lr=0.05, momentum=0.9, weight_decay=1e-4, foreach=True)
        states = ["momentum_buffer"]
    elif kind == "adam":
        ref = torch.optim.Adam(rp, lr=1e-3, foreach=True)
        fus = FusedAdam(fp, lr=1e-3, foreach=True)
        states = ["exp_avg", "exp_avg_sq"]
    else:
        ref = torch.optim.AdamW(rp, lr=1e-3, weight_decay=0.01, foreach=True)
        fus = FusedAdamW(fp, lr=1e-3, weight_decay=0.01, foreach=True)
        states = ["exp_avg", "exp_avg_sq"]
    gen = torch.Generator(device="cuda").manual_seed(1)
    for step in range(4):
        for n, a, b in zip(names, rp, fp):
            if n not in grads:
                a.grad = b.grad = None
                continue
            g = grads[n] * (1.0 + 0.5 * torch.rand((), device="cuda", generator=gen))  # vary per step
            a.grad = g.clone()
            b.grad = g.clone()
        ref.step()
        fus.step()
        bad = []
        for n, a, b in zip(names, rp, fp):
            if not torch.allclose(a, b, rtol=2e-5, atol=1e-7):
                bad.append((step, n, "param", (a - b).abs().max().item()))
            if n not in grads:
                continue
            for k in states:
                sa, sb = ref.state[a][k], fus.state[b][k]
                if not torch.allclose(sa, sb, rtol=2e-5, atol=1e-9):
                    bad.append((step, n, k, (sa - sb).abs().max().item()))
        assert not bad, bad[:8]
    assert fus.fused_steps == 4, "the fused kernel did not run (stock fallback)"


def _trainer(tmp_path, **kw):
    from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer

    c = BaseConfig()
    c.dataset, c.num_class, c.model, c.arch_type, c.use_aux = "cityscapes", 19, "ddrnet", "DDRNet-23", True
    c.synthetic_data, c.synthetic_len, c.synthetic_size = True, 8, (128, 256)
    c.crop_size, c.crop_h, c.crop_w = 128, 128, 256
    c.train_bs, c.val_bs, c.total_epoch = 2, 2, 50
    c.amp_training, c.amp_dtype, c.channels_last = True, "bf16", True
    c.base_workers, c.use_tb, c.save_ckpt, c.load_ckpt, c.use_ema = 0, False, False, False, True
    c.save_dir = str(tmp_path / "save")
    for k, v in kw.items():
        setattr(c, k, v)
    c.init_dependent_config()
    return SegTrainer(c)


def test_trainer_takes_fused_path_and_ema_matches_reference(tmp_path):
    """Trainer-level: the fused step + EMA runs on DDRNet-23 channels-last, and the EMA it writes
    equals the reference formula applied to the model's parameters step by step."""
    tr = _trainer(tmp_path)
    from realtime_semantic_segmentation_pytorch_amd.datasets import DeviceBatches

    data = DeviceBatches(2, (128, 256), 19, 255, device=tr.device, pool=1, channels_last=True, seed=1)
    imgs, masks = data.next()
    ema = {n: p.detach().clone() for n, p in tr.model.named_parameters()}
    for it in range(3):
        tr.train_step(imgs, masks)
        d = tr.ema_model.decay(tr.train_itrs)
        for n, p in tr.model.named_parameters():
            ema[n] = d * ema[n] + (1 - d) * p.detach()
    assert tr.ema_fused and tr.optimizer.fused_steps == 3 and tr.optimizer.last_step_fused
    got = dict(tr.ema_model.ema.named_parameters())
    for n, e in ema.items():
        torch.testing.assert_close(got[n], e, rtol=1e-5, atol=1e-6)


def test_ema_validation_sees_new_weights_after_training(tmp_path):
    """The eval-time caches (bf16 conv weights, BN eval coefficients) must not survive a fused
    optimizer / EMA write: validate, train, validate again == a fresh copy of the EMA model."""
    tr = _trainer(tmp_path, total_epoch=4)
    from realtime_semantic_segmentation_pytorch_amd.datasets import DeviceBatches

    data = DeviceBatches(2, (128, 256), 19, 255, device=tr.device, pool=1, channels_last=True, seed=2)
    imgs, masks = data.next()
    x = imgs[:1]

    def infer(model):
        model.eval()
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            return ops.materialize(model(x)).float()

    for _ in range(2):
        tr.train_step(imgs, masks)
    first = infer(tr.ema_model.ema)
    for _ in range(3):
        tr.train_step(imgs, masks)
    assert tr.optimizer.fused_steps == 5
    second = infer(tr.ema_model.ema)
    fresh = infer(copy.deepcopy(tr.ema_model.ema))
    assert not torch.equal(first, second), "EMA model output did not change after training"
    # a stale cache would serve the weights of `first`: second must sit at bf16-rounding distance
    # from the fresh copy, far closer than first does.  Not bitwise: cached-weight inference and
    # a deep copy differ by bf16 rounding even with every cache invalidated (max |diff| ~1e-3,
    # tools/probe_ema_determinism.py; the round-4 suite hit 1.5e-3 on half the elements)
    d_new, d_old = (second - fresh).norm().item(), (first - fresh).norm().item()
    assert d_new <= 0.25 * d_old, (d_new, d_old)
    # two bf16 ulps at the output's largest magnitude (measured: one ulp, 9.8e-4 at max 0.2)
    torch.testing.assert_close(second, fresh, rtol=0, atol=2 ** -6 * fresh.abs().max().item())


def _shadow_run(shadow_on, monkeypatch, steps=3):
    from realtime_semantic_segmentation_pytorch_amd.models.modules import ConvBNAct
    from realtime_semantic_segmentation_pytorch_amd.ops import conv as conv_mod
    from realtime_semantic_segmentation_pytorch_amd.ops.optim import FusedSGD

    monkeypatch.setattr(conv_mod, "_SHADOW_ON", shadow_on)
    torch.manual_seed(0)
    m = torch.nn.Sequential(ConvBNAct(64, 64, 3), ConvBNAct(64, 128, 3), ConvBNAct(128, 128, 1))
    m = m.cuda().to(memory_format=torch.channels_last).train()
    ops.convert_batchnorm(m)
    opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(steps):
        x = torch.randn(4, 64, 32, 48, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        (y.float() ** 2).mean().backward()
        opt.step()
        assert opt.fused_steps > 0
    torch.cuda.synchronize()
    shadows = {n: conv_mod.shadow_of(p) for n, p in m.named_parameters()}
    return {n: p.detach().clone() for n, p in m.named_parameters()}, shadows, m


def test_weight_shadows_written_by_the_fused_step(monkeypatch):
    """The fused step rewrites the bf16 krsc / crsk copies of every routed conv weight
    (ops/conv.py _Shadow): training with them is bitwise the training with the per-step cast +
    transpose, and after the step they equal the bf16 casts of the updated weights."""
    ref, _, _ = _shadow_run(False, monkeypatch)
    got, shadows, m = _shadow_run(True, monkeypatch)
    for n in ref:
        torch.testing.assert_close(got[n], ref[n], rtol=0, atol=0, msg=n)
    seen = 0
    for n, p in m.named_parameters():
        sh = shadows[n]
        if sh is None:
            continue
        seen += 1
        w16 = p.detach().to(torch.bfloat16)
        assert torch.equal(sh.krsc, w16.permute(0, 2, 3, 1).contiguous()), n
        assert torch.equal(sh.crsk, w16.permute(1, 2, 3, 0).contiguous()), n
    assert seen >= 2


def test_weight_shadow_follows_writes_outside_the_optimizer(monkeypatch):
    """A parameter write the fused step did not make: ``p.copy_`` under no_grad (version bump, as
    ``load_state_dict`` does) is seen by itself; a ``p.data`` write (its own version counter) or a
    collective into the storage is seen after ``ops.invalidate_weight_shadows`` (what
    ``parallel_model`` calls after DDP's initial broadcast).  The next training forward then
    equals the forward of a fresh model holding the new weights."""
    _, _, m = _shadow_run(True, monkeypatch, steps=1)
    torch.manual_seed(5)
    x = torch.randn(4, 64, 32, 48, device="cuda").contiguous(memory_format=torch.channels_last)

    def fwd(mod):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return mod(x).float()

    import copy

    convs = [p for n, p in m.named_parameters() if p.dim() == 4]
    new = [torch.randn_like(p) * p.std() for p in convs]
    with torch.no_grad():
        for p, v in zip(convs, new):
            p.copy_(v)
    fresh = copy.deepcopy(m)
    for p in fresh.parameters():
        p._rtseg_shadow = None
    torch.testing.assert_close(fwd(m), fwd(fresh), rtol=0, atol=0)
    new2 = [torch.randn_like(p) * p.std() for p in convs]
    for p, v in zip(convs, new2):
        p.data.copy_(v)
    assert ops.invalidate_weight_shadows(m.parameters()) >= 2
    fresh2 = copy.deepcopy(m)
    for p in fresh2.parameters():
        p._rtseg_shadow = None
    torch.testing.assert_close(fwd(m), fwd(fresh2), rtol=0, atol=0)
