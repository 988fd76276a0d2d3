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


def check_zoo_hip_matches_torch_path(key, monkeypatch):
    """Eval forward: HIP path == torch path (tight).  Training step (forward, loss, backward): the
    HIP path (channels-last) is scored against a CPU fp64 run of the same step, with two
    yardsticks measured in the same test -- the CPU fp32 run and the GPU torch path in NCHW.

    Measured on MI355X (tools/probe_zoo_gpu_err.py, profiles/r3_zoo_numerics): the channels-last
    torch path is ~1e-2 off fp64 on the pooling models even with frozen BatchNorm (round 3 blamed
    MIOpen's NHWC convs; the round-4 bisection, profiles/r4_numerics, pins it on PyTorch's
    channels-last avg_pool2d backward -- the HIP path runs the same MIOpen convs at 1e-5), so it
    is NOT a usable yardstick (round 2 used it and had to skip 7 models).  Two passes, no skips:
    * frozen BatchNorm (running statistics): every model's whole HIP training path -- convs,
      depth-wise convs, pooling, interpolation, gating, activations, the loss -- must be within
      10x the CPU fp32 error (floor 1e-3);
    * batch-statistics BatchNorm at batch 2: within 4x the better of the two yardsticks, or 1.5x
      the worse, or the flip envelope of a batch-2 BN sign flip (``TRAIN_BN_FLIP_FLOOR``).  Where even CPU fp32 is > 0.1 off fp64 (DFANet, Lite-HRNet, MiniNetV2: BN over a
      handful of values at batch 2, gradients of ~1e8), the step is only checked for finite
      gradients; the frozen pass above still pins their numerics."""
    torch.manual_seed(0)
    cpu = _model(key)
    for mod in cpu.modules():  # CPU and GPU RNG streams differ: compare without dropout
        if isinstance(mod, torch.nn.modules.dropout._DropoutNd):
            mod.p = 0.0
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
    for frozen in (True, False):
        prep = _freeze_bn if frozen else (lambda m: m)
        bn = "frozen-BN" if frozen else "train-BN"
        y_r, l_r, g_r = _run_gpu(prep(copy.deepcopy(cpu).train().double()), x.double(), labels, False, monkeypatch)
        y_c, l_c, g_c = _run_gpu(prep(copy.deepcopy(cpu).train()), x, labels, False, monkeypatch)
        y_h, l_h, g_h = _run_gpu(prep(copy.deepcopy(base).train()), xg, labels.cuda(), False, monkeypatch,
                                 f"{key} {bn} HIP fp32")
        assert g_h.keys() == g_c.keys() == g_r.keys()
        cat = lambda g: torch.cat([g[n].flatten().double().cpu() for n in g_r])  # noqa: E731
        hg, cg = err(cat(g_h), cat(g_r)), err(cat(g_c), cat(g_r))
        assert torch.isfinite(cat(g_h)).all()
        tag = f"{key} {'frozen-BN' if frozen else 'train-BN'}: HIP grad err {hg:.2e}, CPU fp32 {cg:.2e}"
        if frozen:
            assert err(y_h, y_r) <= max(10 * err(y_c, y_r), 1e-4), tag
            assert abs(l_h.item() - l_r.item()) <= max(10 * abs(l_c.item() - l_r.item()), 1e-4 * abs(l_r.item())), tag
            assert hg <= max(10 * cg, 1e-3), tag
            _check_bf16_vs_fp64(key, base, xg, labels, l_r, g_r, cat, err, monkeypatch)
            continue
        if cg > 0.1:
            continue  # ill-conditioned at batch 2 on any path (see docstring); finiteness checked
        nchw = copy.deepcopy(cpu).cuda().train()
        _, l_t, g_t = _run_gpu(nchw, x.cuda(), labels.cuda(), True, monkeypatch, f"{key} {bn} stock fp32 NCHW")
        tg = err(cat(g_t), cat(g_r))
        tag += f", GPU torch NCHW {tg:.2e}"
        print(tag)
        assert abs(l_h.item() - l_r.item()) <= max(4 * min(abs(l_t.item() - l_r.item()), abs(l_c.item() - l_r.item())),
                                                   1e-3 * abs(l_r.item())), tag
        # batch-2 batch statistics make this step ill-conditioned: a BN over 2 values per channel
        # (DDRNet's DAPPM global branch, BiSeNetV2's context block) normalises to +-d/sqrt(d^2 +
        # eps), and where d is rounding-sized the sign -- which sample passes its ReLU -- flips
        # with the last bits of upstream sums.  Such a flip moves the whole gradient by
        # ~3.5e-3 (DDRNet) in ANY path: on identical inputs the stock GPU path gave 1.5e-5 in one
        # process and 3.46e-3 in the next, the HIP path 1.2e-5 or 3.47e-3, and at batch 4 even
        # CPU fp32 shows 3.05e-3 (tools/probe_param_err.py, profiles/r5_numerics).  So the HIP
        # path must be within 4x the better yardstick, or 1.5x the worse one, or the measured
        # flip envelope; the frozen-BN pass above pins every kernel's precision without flips.
        assert hg <= max(4 * min(tg, cg), 1.5 * max(tg, cg), TRAIN_BN_FLIP_FLOOR), tag


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


# a sign flip of a batch-2 BatchNorm over 2 values (see check_zoo_hip_matches_torch_path): the
# gradient error one flip leaves on DDRNet-23, measured on the stock GPU path too (3.46e-3)
TRAIN_BN_FLIP_FLOOR = 4e-3

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
