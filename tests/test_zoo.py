"""Whole-zoo training-path tests.

CPU: every registered model runs a train step through the trainer's path
(deferred final upsample -> fused-loss formulation -> backward) and the deferred
logits materialise to exactly the model's normal output.

GPU (in the pytest process): every model in fp32 channels-last runs forward + loss + backward
on the HIP kernels, scored against a CPU fp64 run with the CPU fp32 run and the GPU NCHW torch
path as yardsticks, with frozen and with batch-statistics BatchNorm; the production bf16 path
(autocast, channels-last, MFMA convs) is scored against the same fp64 frozen-BN step, bounded by
stock bf16's distance (``check_zoo_hip_matches_torch_path``).  A second GPU test runs the
production configuration with OHEM and aux heads and checks for finite loss/gradients.
"""
import copy

import pytest
import torch

import _faultlog

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
from realtime_semantic_segmentation_pytorch_amd.core.loss import SegCELoss
from realtime_semantic_segmentation_pytorch_amd.models import (AUX_MODELS, DETAIL_HEAD_MODELS, MODEL_HUB,
                                                               get_model)
from realtime_semantic_segmentation_pytorch_amd.ops.interp import DeferredLogits

KEYS = sorted(MODEL_HUB)
HW = (128, 256)


def _model(key, use_aux=False):
    c = BaseConfig()
    c.model, c.num_class = key, 19
    c.use_aux = use_aux and key in AUX_MODELS
    c.use_detail_head = False
    torch.manual_seed(0)
    return get_model(c)


def _main(out):
    return out[0] if isinstance(out, (tuple, list)) else out


def _forward(m, x):
    kw = {"is_training": True} if m.training else {}
    return m(x, **kw)


@pytest.mark.parametrize("key", KEYS)
def test_train_step_with_deferred_upsample_cpu(key):
    m = _model(key, use_aux=True).train()
    x = torch.randn(2, 3, *HW)
    labels = torch.randint(0, 19, (2, *HW))
    loss_fn = SegCELoss(ops.MODE_OHEM, 0.7)
    with ops.defer_final_upsample():
        out = _forward(m, x)
    main = _main(out)
    assert main.shape == (2, 19, *HW)
    loss = loss_fn(main, labels)
    if isinstance(out, (tuple, list)) and len(out) > 1:
        for a in out[1] if isinstance(out[1], (list, tuple)) else [out[1]]:
            loss = loss + loss_fn.aux(a, labels)
    loss.backward()
    assert torch.isfinite(loss)
    grads = [p.grad for p in m.parameters() if p.requires_grad]
    assert sum(g is not None for g in grads) >= 0.9 * len(grads)
    assert all(torch.isfinite(g).all() for g in grads if g is not None)


@pytest.mark.parametrize("key", KEYS)
def test_deferred_logits_materialize_to_model_output_cpu(key):
    m = _model(key).eval()
    x = torch.randn(1, 3, *HW)
    ref = _main(m(x))
    with ops.defer_final_upsample():
        out = _main(m(x))
    got = out.materialize() if isinstance(out, DeferredLogits) else out
    torch.testing.assert_close(got, ref, atol=1e-5, rtol=1e-5)


def _run_gpu(m, x, labels, disable_hip, monkeypatch, phase=None):
    if phase is not None:  # survives an abort (tests/_faultlog.py)
        _faultlog.write(f"  phase {phase}")
    if disable_hip:
        monkeypatch.setenv("RTSEG_DISABLE_HIP", "1")
    else:
        monkeypatch.delenv("RTSEG_DISABLE_HIP", raising=False)
    torch.manual_seed(123)
    with ops.defer_final_upsample():
        out = _main(_forward(m, x))
    loss = SegCELoss(ops.MODE_MEAN)(out, labels)
    loss.backward()
    full = out.materialize() if isinstance(out, DeferredLogits) else out
    grads = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    monkeypatch.delenv("RTSEG_DISABLE_HIP", raising=False)
    return full.detach(), loss.detach(), grads


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-6)).item()


def _freeze_bn(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
            mod.eval()
    return m


# A training-mode BatchNorm whose per-channel population N*H*W is below this runs on its running
# statistics in the train-BN numerics pass (all paths identically).  Such a BN normalises a handful
# of values to +-d/sqrt(d^2 + eps); where d is rounding-sized the sign -- which value passes the
# next ReLU -- flips with the last bits of upstream sums, in ANY path (AGLNet's 1-channel pyramid on
# 4 x 8 maps, DDRNet's DAPPM global branch over 2 values).  tools/probe_bn_population.py: at 1024
# AGLNet's CPU fp32 error drops 6.8e-3 -> 4.2e-4, ContextNet 3.3e-2 -> 4e-6, FastSCNN 8e-3 -> 2e-6;
# other discrete events remain (see check_zoo_hip_matches_torch_path), so this alone is not a
# criterion (profiles/r6_zoo_numerics).
SMALL_BN_POPULATION = 1024


def bn_populations(m, x):
    """{module name: per-channel population N*H*W} of every BatchNorm of ``m`` in a training
    forward of ``x`` on the CPU (smallest over repeated calls)."""
    m = copy.deepcopy(m).train()
    pops, hooks = {}, []
    for name, mod in m.named_modules():
        if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
            def pre(mod_, args, name=name):
                t = args[0]
                p = t.numel() // t.shape[1]
                pops[name] = min(pops.get(name, p), p)
            hooks.append(mod.register_forward_pre_hook(pre))
    with torch.no_grad():
        _forward(m, x)
    for h in hooks:
        h.remove()
    return pops


def freeze_small_bn(m, pops, threshold=SMALL_BN_POPULATION):
    """Put every BatchNorm of ``m`` whose population (``bn_populations``) is below ``threshold``
    in eval mode (running statistics) -- after ``m.train()``."""
    mods = dict(m.named_modules())
    for name, p in pops.items():
        if p < threshold:
            mods[name].eval()
    return m


def _no_dropout(m):
    for mod in m.modules():  # CPU and GPU RNG streams differ: compare without dropout
        if isinstance(mod, torch.nn.modules.dropout._DropoutNd):
            mod.p = 0.0
    return m


def _grad_err(g, r):
    a = torch.cat([g[n].flatten().double() for n in r])
    b = torch.cat([r[n].flatten().double() for n in r])
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _cpu_grads(m, x, labels):
    with ops.defer_final_upsample():
        o = _main(_forward(m, x))
    SegCELoss(ops.MODE_MEAN)(o, labels).backward()
    return {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}


def perturb_ulp(m, seed):
    """Multiply every parameter of fp32 model ``m`` by (1 + 2^-24 * N(0, 1)) -- a rounding-sized
    change, so the step's distance to the unperturbed fp64 step is one more independent draw of
    fp32 rounding noise (through the same chaotic sign decisions)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in m.parameters():
            p.mul_(1 + 2.0 ** -24 * torch.randn(p.shape, generator=g, dtype=torch.float64).to(p.dtype))
    return m


def cpu_fp32_vs_fp64_train_bn(key, x, labels, threshold=SMALL_BN_POPULATION, draws=0):
    """CPU fp32 whole-model gradient error vs CPU fp64 of one batch-statistics training step with
    the small-population BatchNorms frozen; with ``draws`` > 0 a list: the plain fp32 error then
    ``draws`` errors of ulp-perturbed fp32 models (``perturb_ulp``)."""
    torch.manual_seed(0)
    cpu = _no_dropout(_model(key))
    pops = bn_populations(cpu, x)
    prep = lambda dt: freeze_small_bn(copy.deepcopy(cpu).train().to(dt), pops, threshold)  # noqa: E731
    ref = _cpu_grads(prep(torch.float64), x.double(), labels)
    errs = [_grad_err(_cpu_grads(prep(torch.float32), x, labels), ref)]
    for d in range(draws):
        errs.append(_grad_err(_cpu_grads(perturb_ulp(prep(torch.float32), d + 1), x, labels), ref))
    return errs if draws else errs[0]


def test_small_bn_freeze_covers_the_batch2_flip_sites_cpu():
    """The sites behind the round-5 driver failure (AGLNet's 1-channel ConvBNAct pyramid, reference
    models/aglnet.py:99-104) and DDRNet's DAPPM global branch run on running statistics in the
    train-BN pass; the full-resolution BNs keep batch statistics."""
    x = torch.randn(2, 3, *HW)
    for key in ("aglnet", "ddrnet"):
        m = _model(key)
        pops = bn_populations(m, x)
        assert min(pops.values()) < 64 and max(pops.values()) >= 2 * (HW[0] // 2) * (HW[1] // 2) // 4
        f = freeze_small_bn(copy.deepcopy(m).train(), pops)
        mods = dict(f.named_modules())
        assert all(mods[n].training == (p >= SMALL_BN_POPULATION) for n, p in pops.items())


@pytest.mark.parametrize("key", ["aglnet", "ddrnet", "lite_hrnet"])
def test_train_bn_envelope_accepts_a_rounding_draw_cpu(key):
    """The GPU train-BN criterion on the CPU: more ulp-perturbed fp32 runs (stand-ins for a correct
    HIP path and its re-draws: rounding noise only) land within ``ZOO_ENVELOPE_X`` x the envelope of the
    plain fp32 run and ``ZOO_CPU_DRAWS`` draws -- including on Lite-HRNet, where every draw is
    ~5e-3 off fp64, and on DDRNet-23, whose draws are 2.7e-6 or, when the ReLU after a 1024-value BN
    (conv5.high_conv1) flips one element, 1.4e-3 -- while a 5 % systematic gradient error (a bug) would not."""
    torch.manual_seed(0)
    x = torch.randn(2, 3, *HW)
    labels = torch.randint(0, 19, (2, *HW))
    errs = cpu_fp32_vs_fp64_train_bn(key, x, labels, draws=ZOO_CPU_DRAWS + 1 + ZOO_HIP_DRAWS)
    env, cand = errs[:ZOO_CPU_DRAWS + 1], errs[ZOO_CPU_DRAWS + 1:]
    assert min(cand) <= ZOO_ENVELOPE_X * max(env), (cand, env)
    assert 5e-2 > ZOO_ENVELOPE_X * max(env), env  # a bug of 5 % would fail


def check_zoo_hip_matches_torch_path(key, monkeypatch):
    """Eval forward: HIP path == torch path (tight).  Training step (forward, loss, backward): the
    HIP path (channels-last) is scored against a CPU fp64 run of the same step.

    Measured on MI355X (tools/probe_zoo_gpu_err.py, profiles/r3_zoo_numerics): the channels-last
    torch path is ~1e-2 off fp64 on the pooling models even with frozen BatchNorm (round 4,
    profiles/r4_numerics: PyTorch's channels-last avg_pool2d backward), so it is NOT a yardstick.
    Two passes, no skips:
    * frozen BatchNorm (running statistics): every model's whole HIP training path -- convs,
      depth-wise convs, pooling, interpolation, gating, activations, the loss -- must be within
      10x the CPU fp32 error (floor 1e-3), plus the production bf16 path (``_check_bf16_vs_fp64``);
    * batch-statistics BatchNorm at batch 2.  This step is chaotic on every path: a BN over a
      handful of values normalises to +-d/sqrt(d^2 + eps), and wherever a rounding-sized change
      decides a discrete event (that sign, a ReLU on a pooled vector, a max-pool winner) the whole
      gradient jumps.  Measured on CPU (tools/probe_bn_population.py, profiles/r6_zoo_numerics):
      fp32-vs-fp64 errors of ulp-perturbed copies of ONE model are bimodal (DDRNet 2.7e-6 or
      1.4e-3; Lite-HRNet 4e-3..8e-3), so any single-draw yardstick flips.  Hence:
      - BatchNorms whose per-channel population is below ``SMALL_BN_POPULATION`` run on running
        statistics in every path (the batch-2 sign flips: AGLNet's 1-channel pyramid on 4 x 8
        maps, reference models/aglnet.py:99-104);
      - the envelope is measured in the test: CPU fp32 plus ``ZOO_CPU_DRAWS`` ulp-perturbed fp32
        draws (``perturb_ulp``) and the GPU NCHW stock path;
      - the HIP path (plus up to ``ZOO_HIP_DRAWS`` ulp-perturbed re-runs, taken only while it is
        outside) must land within ``ZOO_ENVELOPE_X`` x the envelope's largest error, or within
        ``ZOO_SAME_LAYOUT_X`` x the stock path run on the same channels-last tensors (which shares
        MIOpen's channels-last fp32 convs: SegNet is 3.0e-2 off fp64 on both, profiles/r6_zoo_numerics).
      A kernel bug is systematic: it survives every HIP draw.  A flip does not."""
    monkeypatch.setenv("RTSEG_TUNE_FIXED", "1")  # conv choices by rule, not timing (reproducible)
    torch.manual_seed(0)
    cpu = _no_dropout(_model(key))
    x = torch.randn(2, 3, *HW)
    labels = torch.randint(0, 19, (2, *HW))
    base = copy.deepcopy(cpu).cuda().to(memory_format=torch.channels_last)
    xg = x.cuda().contiguous(memory_format=torch.channels_last)
    # eval: deterministic, tight
    ev = copy.deepcopy(base).eval()
    with torch.no_grad():
        monkeypatch.delenv("RTSEG_DISABLE_HIP", raising=False)
        e_h = _main(ev(xg)).float()
        monkeypatch.setenv("RTSEG_DISABLE_HIP", "1")
        e_t = _main(ev(xg)).float()
        monkeypatch.delenv("RTSEG_DISABLE_HIP", raising=False)
    assert _rel(e_h, e_t) < 2e-5
    err = lambda a, b: ((a.double().cpu() - b.double().cpu()).norm() / (b.double().cpu().norm() + 1e-30)).item()  # noqa: E731
    pops = bn_populations(cpu, x)
    for frozen in (True, False):
        prep = _freeze_bn if frozen else (lambda m: freeze_small_bn(m, pops))
        bn = "frozen-BN" if frozen else "train-BN"
        y_r, l_r, g_r = _run_gpu(prep(copy.deepcopy(cpu).train().double()), x.double(), labels, False, monkeypatch)
        y_c, l_c, g_c = _run_gpu(prep(copy.deepcopy(cpu).train()), x, labels, False, monkeypatch)
        y_h, l_h, g_h = _run_gpu(prep(copy.deepcopy(base).train()), xg, labels.cuda(), False, monkeypatch,
                                 f"{key} {bn} HIP fp32")
        assert g_h.keys() == g_c.keys() == g_r.keys()
        cat = lambda g: torch.cat([g[n].flatten().double().cpu() for n in g_r])  # noqa: E731
        hg, cg = err(cat(g_h), cat(g_r)), err(cat(g_c), cat(g_r))
        assert torch.isfinite(cat(g_h)).all()
        tag = f"{key} {bn}: HIP grad err {hg:.2e}, CPU fp32 {cg:.2e}"
        if frozen:
            assert err(y_h, y_r) <= max(10 * err(y_c, y_r), 1e-4), tag
            assert abs(l_h.item() - l_r.item()) <= max(10 * abs(l_c.item() - l_r.item()), 1e-4 * abs(l_r.item())), tag
            assert hg <= max(10 * cg, 1e-3), tag
            _check_bf16_vs_fp64(key, base, xg, labels, l_r, g_r, cat, err, monkeypatch)
            continue
        nchw = prep(copy.deepcopy(cpu).cuda().train())
        _, l_t, g_t = _run_gpu(nchw, x.cuda(), labels.cuda(), True, monkeypatch, f"{key} {bn} stock fp32 NCHW")
        env = [cg, err(cat(g_t), cat(g_r))]
        lenv = [abs(l_c.item() - l_r.item()), abs(l_t.item() - l_r.item())]
        for d in range(ZOO_CPU_DRAWS):
            _, l_d, g_d = _run_gpu(perturb_ulp(prep(copy.deepcopy(cpu).train()), d + 1), x, labels, False,
                                   monkeypatch)
            env.append(err(cat(g_d), cat(g_r)))
            lenv.append(abs(l_d.item() - l_r.item()))
        # the stock path on the SAME channels-last tensors: it shares MIOpen's channels-last fp32
        # convs with the HIP path, whose rounding moves discrete decisions the NCHW / CPU runs do not
        # (SegNet: max-unpool positions after a ReLU, 3.0e-2 on both paths, profiles/r6_zoo_numerics)
        _, l_s, g_s = _run_gpu(prep(copy.deepcopy(base).train()), xg, labels.cuda(), True, monkeypatch,
                               f"{key} {bn} stock fp32 channels-last")
        sg, sl = err(cat(g_s), cat(g_r)), abs(l_s.item() - l_r.item())
        hip = [hg]
        lh = abs(l_h.item() - l_r.item())
        # within the rounding envelope, or no worse than stock PyTorch on the same layout (whose own
        # avg_pool2d backward is ~1e-2 off on the pooling models: that clause only ever adds a pass
        # where the HIP path matches stock)
        bound = max(ZOO_ENVELOPE_X * max(env), ZOO_SAME_LAYOUT_X * sg)
        lbound = max(ZOO_ENVELOPE_X * max(max(lenv), 1e-7 * abs(l_r.item())), ZOO_SAME_LAYOUT_X * sl)
        for d in range(ZOO_HIP_DRAWS):
            if min(hip) <= bound and lh <= lbound:
                break
            m = perturb_ulp(prep(copy.deepcopy(cpu).train()), 100 + d).cuda().to(memory_format=torch.channels_last)
            _, l_d, g_d = _run_gpu(m, xg, labels.cuda(), False, monkeypatch, f"{key} {bn} HIP fp32 draw {d + 1}")
            hip.append(err(cat(g_d), cat(g_r)))
            lh = min(lh, abs(l_d.item() - l_r.item()))
        tag = (f"{key} {bn}: HIP grad err {', '.join(f'{h:.2e}' for h in hip)}; envelope (CPU fp32, GPU NCHW, "
               f"{ZOO_CPU_DRAWS} CPU draws) {', '.join(f'{e:.2e}' for e in env)}; stock channels-last {sg:.2e}; "
               f"loss err {lh:.2e} (envelope max {max(lenv):.2e}, stock channels-last {sl:.2e})")
        print(tag)
        assert min(hip) <= bound, tag
        assert lh <= lbound, tag


def _run_gpu_bf16(m, x, labels, disable_hip, monkeypatch, phase=None):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        return _run_gpu(m, x, labels, disable_hip, monkeypatch, phase)


def _check_bf16_vs_fp64(key, base, xg, labels, l_r, g_r, cat, err, monkeypatch):
    """The PRODUCTION path (bf16 autocast, channels-last, every HIP kernel incl. the MFMA convs,
    depth-wise / BN / pooling / gating kernels) against the same frozen-BN training step in fp64
    on the CPU, bounded by stock PyTorch bf16's own distance to fp64 on that step (the criterion
    of tests/test_train_numerics_gpu.py): the whole-model gradient error and the loss error.
    Frozen BatchNorm keeps batch-statistics amplification out, so the errors measure rounding."""
    lg = labels.cuda()
    _, l_s, g_s = _run_gpu_bf16(_freeze_bn(copy.deepcopy(base).train()), xg, lg, True, monkeypatch,
                                f"{key} frozen-BN stock bf16")
    _, l_b, g_b = _run_gpu_bf16(_freeze_bn(copy.deepcopy(base).train()), xg, lg, False, monkeypatch,
                                f"{key} frozen-BN HIP bf16")
    assert g_b.keys() == g_r.keys() == g_s.keys(), key
    sg, bg = err(cat(g_s), cat(g_r)), err(cat(g_b), cat(g_r))
    sl, bl = abs(l_s.item() - l_r.item()), abs(l_b.item() - l_r.item())
    tag = f"{key} bf16 frozen-BN: HIP grad err {bg:.2e} (stock {sg:.2e}), loss err {bl:.2e} (stock {sl:.2e})"
    print(tag)
    assert torch.isfinite(cat(g_b)).all(), tag
    assert bg <= max(ZOO_BF16_GRAD_SLACK * sg, ZOO_BF16_GRAD_FLOOR), tag
    assert bl <= max(ZOO_BF16_LOSS_SLACK * sl, 2e-3 * abs(l_r.item())), tag


# the train-BN envelope (check_zoo_hip_matches_torch_path): ulp-perturbed CPU fp32 draws measured
# per test, the factor on the envelope's largest error, and HIP re-draws taken while outside it
ZOO_CPU_DRAWS, ZOO_ENVELOPE_X, ZOO_HIP_DRAWS = 3, 2.0, 2
ZOO_SAME_LAYOUT_X = 1.5  # ... or within this factor of the stock path on the same channels-last tensors

# HIP bf16 vs stock bf16 distance to fp64 (frozen BN, 128 x 256, batch 2).  Round 5 on MI355X: HIP
# / stock between 0.14 (SwiftNet) and 1.14 (ENet), smallest stock 4.6e-3 (FastSCNN); the floor
# (2e-2 until round 4) only covers stock's run-to-run spread below 5e-3.
ZOO_BF16_GRAD_SLACK, ZOO_BF16_GRAD_FLOOR, ZOO_BF16_LOSS_SLACK = 1.5, 5e-3, 2.0


@pytest.mark.gpu
@pytest.mark.parametrize("key", KEYS)
def test_zoo_hip_matches_torch_path_gpu(key, monkeypatch):
    check_zoo_hip_matches_torch_path(key, monkeypatch)


@pytest.mark.gpu
@pytest.mark.parametrize("key", KEYS)
def test_zoo_bf16_channels_last_train_step_gpu(key):
    check_zoo_bf16_channels_last_train_step(key)


def check_zoo_bf16_channels_last_train_step(key):
    m = _model(key, use_aux=True).cuda().to(memory_format=torch.channels_last).train()
    x = torch.randn(2, 3, *HW, device="cuda").contiguous(memory_format=torch.channels_last)
    labels = torch.randint(0, 19, (2, *HW), device="cuda", dtype=torch.uint8)
    loss_fn = SegCELoss(ops.MODE_OHEM, 0.7)
    with torch.autocast("cuda", dtype=torch.bfloat16), ops.defer_final_upsample():
        out = _forward(m, x)
        loss = loss_fn(_main(out), labels)
        if isinstance(out, (tuple, list)) and len(out) > 1:
            for a in out[1] if isinstance(out[1], (list, tuple)) else [out[1]]:
                loss = loss + loss_fn.aux(a, labels)
    loss.backward()
    assert torch.isfinite(loss)
    assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)
