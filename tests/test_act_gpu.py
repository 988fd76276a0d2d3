"""HIP activation family (act.hip) against PyTorch fp32 autograd: forward, input gradient and the
PReLU weight gradient, channels-last and contiguous, fp32 / bf16.  Reference:
models/modules.py:111-131 (Activation hub)."""
import pytest
import torch
import torch.nn as nn

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.ops import act as A

pytestmark = pytest.mark.gpu

MODULES = [lambda c: nn.PReLU(), lambda c: nn.PReLU(c), lambda c: nn.LeakyReLU(0.1), lambda c: nn.ELU(0.7),
           lambda c: nn.CELU(1.3), lambda c: nn.SELU(), lambda c: nn.Hardswish(), lambda c: nn.Hardtanh(-1.5, 2.0),
           lambda c: nn.SiLU(), lambda c: nn.Sigmoid(), lambda c: nn.Tanh(), lambda c: nn.GELU(),
           lambda c: nn.GELU(approximate="tanh")]


@pytest.mark.parametrize("mi", range(len(MODULES)))
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [True, False])
@pytest.mark.parametrize("shape", [(2, 24, 17, 33), (3, 64, 32, 40)])
def test_activation_matches_torch(mi, dtype, cl, shape):
    assert ops.load()
    torch.manual_seed(mi)
    ref = MODULES[mi](shape[1]).cuda()
    if isinstance(ref, nn.PReLU):
        with torch.no_grad():
            ref.weight.uniform_(-0.5, 0.5)
    hip = A.convert_activations(MODULES[mi](shape[1]).cuda())
    hip.load_state_dict(ref.state_dict())
    x = (torch.randn(shape, device="cuda") * 3).to(dtype)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    g = torch.randn(shape, device="cuda").to(dtype)
    xr = x.float().detach().requires_grad_(True)
    yr = ref(xr)
    yr.backward(g.float())
    xh = x.detach().requires_grad_(True)
    yh = hip(xh)
    yh.backward(g)
    tol = dict(atol=1e-5, rtol=1e-5) if dtype == torch.float32 else dict(atol=2e-2, rtol=2e-2)
    assert yh.dtype == dtype and yh.shape == yr.shape
    assert torch.allclose(yh.float(), yr, **tol)
    d = (xh.grad.float() - xr.grad).abs()
    bad = d > tol["atol"] + tol["rtol"] * xr.grad.abs()
    assert not bad.any(), f"{int(bad.sum())} bad, e.g. x={x.float()[bad][:4].tolist()} d={d[bad][:4].tolist()}"
    if isinstance(ref, nn.PReLU):
        gw, gr = hip.weight.grad, ref.weight.grad
        assert torch.allclose(gw, gr, atol=1e-3 * gr.abs().max().item() + 1e-4, rtol=1e-3 if dtype == torch.float32 else 2e-2)


def test_prelu_weight_grad_is_deterministic():
    m = A.convert_activations(nn.PReLU(64).cuda())
    x = torch.randn(4, 64, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    g = torch.randn_like(x)
    grads = []
    for _ in range(2):
        m.weight.grad = None
        m(x.requires_grad_(False)).backward(g)
        grads.append(m.weight.grad.clone())
    assert torch.equal(grads[0], grads[1])


def test_zoo_model_trains_through_hip_activations():
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.models import get_model

    cfg = BaseConfig()
    cfg.model, cfg.num_class = "enet", 19
    model = get_model(cfg).cuda().to(memory_format=torch.channels_last).train()
    assert any(isinstance(m, A._HipAct) for m in model.modules())
    x = torch.randn(2, 3, 128, 256, device="cuda").contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = model(x)
    y.float().square().mean().backward()
    prelus = [m for m in model.modules() if isinstance(m, nn.PReLU)]
    assert prelus and all(p.weight.grad is not None and torch.isfinite(p.weight.grad).all() for p in prelus)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [False, True])
@pytest.mark.parametrize("c", [16, 19, 64])
def test_bn_prelu_eval_fused(dtype, cl, c):
    """Inference BN + per-channel PReLU as one pass (ops/bn.py _bn_prelu_eval -> bn_prelu_fwd)
    against BatchNorm2d.eval() then PReLU in fp32; and through a ConvBNAct module tail."""
    import torch.nn as nn

    from realtime_semantic_segmentation_pytorch_amd import ops
    from realtime_semantic_segmentation_pytorch_amd.models.modules import ConvBNAct
    from realtime_semantic_segmentation_pytorch_amd.ops import bn as bn_mod

    assert ops.load()
    torch.manual_seed(c)
    bn = nn.BatchNorm2d(c).cuda().eval()
    pr = nn.PReLU(c).cuda()
    with torch.no_grad():
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
        pr.weight.uniform_(0.05, 0.4)
    x = torch.randn(2, c, 17, 30, device="cuda").to(dtype)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    _, ss = bn_mod.eval_coeffs(bn)
    with torch.no_grad():
        y = torch.ops.rtseg.bn_prelu_fwd(x, pr.weight.contiguous(), ss)
        ref = pr(bn(x.float()))
    tol = dict(rtol=1e-5, atol=1e-5) if dtype == torch.float32 else dict(rtol=2 ** -8, atol=1e-2)
    torch.testing.assert_close(y.float(), ref, **tol)
    assert y.is_contiguous(memory_format=torch.channels_last) == cl or not cl

    m = ops.convert_batchnorm(ConvBNAct(c, c, 3, act_type="prelu")).cuda().eval()
    with torch.no_grad():
        m[1].running_mean.uniform_(-0.5, 0.5)
        m[1].running_var.uniform_(0.5, 2.0)
    before = bn_mod.BN_PRELU_FUSED[0]
    with torch.no_grad():
        got = m(x.float())
    assert bn_mod.BN_PRELU_FUSED[0] > before
    with torch.no_grad():
        conv_out = torch.nn.functional.conv2d(x.float(), m[0].weight, m[0].bias, 1, 1)
        want = torch.nn.functional.prelu(torch.nn.functional.batch_norm(
            conv_out, m[1].running_mean, m[1].running_var, m[1].weight, m[1].bias, False, 0.0, m[1].eps),
            m[2].activation.weight)  # scalar PReLU (the ConvBNAct default): expanded per channel
    torch.testing.assert_close(got.float(), want, rtol=1e-4, atol=1e-4)
