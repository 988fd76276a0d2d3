"""Single-GPU BN backward overlap (ops/bn.py bn_bwd_early): a BN whose output feeds a routed conv
runs its whole backward on a side stream, started right after that conv's data gradient, beside
the conv's weight gradient.  The gradients must be the bits of the one-stream path (same kernels,
same order per stream), the early results must actually be used, and a BN output with a second
consumer must fall back (and not be issued again).  (Opt-in, RTSEG_BN_OVERLAP=1: it measured slower
on DDRNet-23, profiles/r6_negative; the tests switch it on.)"""
import pytest
import torch

from realtime_semantic_segmentation_pytorch_amd import ops

pytestmark = pytest.mark.gpu


def _grads(monkeypatch, on, model_fn, x, gy):
    from realtime_semantic_segmentation_pytorch_amd.ops import bn as bn_mod

    monkeypatch.setattr(bn_mod, "_OVERLAP", on)
    net = model_fn()
    used0 = bn_mod.EARLY_USED[0]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = net(x)
    (y.float() * gy).sum().backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.float().clone() for n, p in net.named_parameters() if p.grad is not None}
    return grads, bn_mod.EARLY_USED[0] - used0, net


def test_rb_chain_bitwise_and_used(monkeypatch):
    from realtime_semantic_segmentation_pytorch_amd.models.ddrnet import RB

    assert ops.load()

    def make():
        torch.manual_seed(0)
        net = ops.convert_batchnorm(torch.nn.Sequential(RB(128, 128), RB(128, 128))).cuda()
        return net.to(memory_format=torch.channels_last).train()

    x = torch.randn(4, 128, 48, 80, device="cuda").contiguous(memory_format=torch.channels_last)
    gy = torch.randn(4, 128, 48, 80, device="cuda")
    g_off, used_off, _ = _grads(monkeypatch, False, make, x, gy)
    g_on, used_on, _ = _grads(monkeypatch, True, make, x, gy)
    assert used_off == 0 and used_on >= 2  # each RB's conv1 -> BN -> ReLU -> conv2
    for n, g in g_off.items():
        assert torch.equal(g_on[n], g), n


def test_second_consumer_falls_back(monkeypatch):
    """conv -> BN -> ReLU whose output feeds a routed conv AND a sum: the BN gradient is a sum,
    so the early results are discarded, the result equals the one-stream path, and the site is
    marked so it is not issued again."""
    from realtime_semantic_segmentation_pytorch_amd.models.modules import ConvBNAct
    from realtime_semantic_segmentation_pytorch_amd.ops import bn as bn_mod

    assert ops.load()

    class Two(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = ConvBNAct(64, 64, 3)
            self.b = ConvBNAct(64, 64, 3)

        def forward(self, x):
            h = self.a(x)
            return self.b(h) + 0.5 * h

    def make():
        torch.manual_seed(1)
        return ops.convert_batchnorm(Two()).cuda().to(memory_format=torch.channels_last).train()

    x = torch.randn(2, 64, 40, 56, device="cuda").contiguous(memory_format=torch.channels_last)
    gy = torch.randn(2, 64, 40, 56, device="cuda")
    g_off, _, _ = _grads(monkeypatch, False, make, x, gy)
    issued0 = bn_mod.EARLY_OVERLAPPED[0]
    g_on, used, net = _grads(monkeypatch, True, make, x, gy)
    for n, g in g_off.items():
        assert torch.equal(g_on[n], g), n
    bn_a = [m for m in net.a.modules() if isinstance(m, torch.nn.BatchNorm2d)][0]
    if bn_mod.EARLY_OVERLAPPED[0] > issued0:  # issued for a's BN, then rejected
        assert getattr(bn_a, "_rtseg_no_early", False)
