"""SyncBN backward all-reduce issued early from the consumer conv (ops.bn.syncbn_bwd_early) at a
site whose BN output has TWO consumers: a routed conv and a second op, ordered so the conv's data
gradient reaches the BN node first.  The early reduction then covers only the conv's part of the
gradient; autograd adds the second consumer's gradient afterwards -- in place into the conv's dx
when nothing else holds it.  The BN backward must notice (``_same_grad``: tensor identity + version
counter, with the early record holding a reference so the add cannot be in place) and reduce the
summed gradient itself.

2 ranks over gloo sharing the GPU (RCCL needs one GPU per rank).  Per rank: the input gradient and
the BN weight / bias gradients with early issuing ON equal those with it OFF (bitwise: the same
kernels reduce the same summed gradient), the early all-reduce was issued and then rejected, and
the site never issues early again.  Both are checked against one CPU fp64 process running the
concatenated batch through plain BatchNorm (bf16 MFMA convs: 2e-2 relative).
Reference wiring: utils/parallel.py:34-43 (torch SyncBatchNorm under DDP).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn as nn

pytestmark = pytest.mark.gpu

N, C, H, W = 2, 64, 16, 24


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    g = torch.Generator().manual_seed(5)
    torch.manual_seed(5)
    conv0 = nn.Conv2d(C, C, 3, 1, 1, bias=False)
    conv1 = nn.Conv2d(C, C, 3, 1, 1, bias=False)
    bn = nn.BatchNorm2d(C)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    x = torch.randn(2 * N, C, H, W, generator=g)
    g1 = torch.randn(2 * N, C, H, W, generator=g)
    g2 = torch.randn(2 * N, C, H, W, generator=g)
    # bf16-representable inputs and weights: the fp64 reference sees what the GPU path sees
    rb = lambda t: t.detach().to(torch.bfloat16).double()  # noqa: E731
    return {"w0": rb(conv0.weight), "w1": rb(conv1.weight), "gamma": bn.weight.detach().double(),
            "beta": bn.bias.detach().double(), "x": rb(x), "g1": g1.double(), "g2": g2.double()}


def _reference(d):
    """One process, fp64, the concatenated batch: dx of conv0's input, dgamma, dbeta."""
    x = d["x"].clone().requires_grad_(True)
    gamma = d["gamma"].clone().requires_grad_(True)
    beta = d["beta"].clone().requires_grad_(True)
    z = torch.nn.functional.conv2d(x, d["w0"], padding=1)
    y = torch.relu(torch.nn.functional.batch_norm(z, None, None, gamma, beta, True, 0.1, 1e-5))
    loss = (y * d["g2"]).sum() + (torch.nn.functional.conv2d(y, d["w1"], padding=1) * d["g1"]).sum()
    loss.backward()
    return x.grad, gamma.grad, beta.grad


def _run(rank, world, port, out):
    for k in ("RTSEG_DISABLE_HIP", "RTSEG_CONV_MFMA", "RTSEG_HIP_OFF"):
        os.environ.pop(k, None)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from realtime_semantic_segmentation_pytorch_amd import ops
    from realtime_semantic_segmentation_pytorch_amd.ops import bn as bn_mod
    from realtime_semantic_segmentation_pytorch_amd.ops.conv import RoutedConv2d

    assert ops.load()
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = _data()
    sl = slice(rank * N, (rank + 1) * N)
    cl = dict(memory_format=torch.channels_last)
    res = {}
    for early in (True, False):
        conv0 = nn.Conv2d(C, C, 3, 1, 1, bias=False)
        conv1 = RoutedConv2d(C, C, 3, 1, 1, bias=False)
        bn = nn.SyncBatchNorm(C)
        with torch.no_grad():
            conv0.weight.copy_(d["w0"])
            conv1.weight.copy_(d["w1"])
            bn.weight.copy_(d["gamma"])
            bn.bias.copy_(d["beta"])
        conv0, conv1, bn = (m.cuda().to(**cl).train() for m in (conv0, conv1, bn))
        if not early:
            bn._rtseg_no_early = True
        x = d["x"][sl].float().cuda().to(torch.bfloat16).contiguous(**cl).requires_grad_(True)
        g1 = d["g1"][sl].float().cuda()
        g2 = d["g2"][sl].float().cuda()
        issued = bn_mod.EARLY_ISSUED[0]
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = ops.conv_bn_act(x, conv0, bn, "relu")
            assert getattr(y.grad_fn, "pg", None) is not None  # the HIP SyncBN node (multi-rank)
            z2 = (y.float() * g2).sum()  # created first: its backward runs after the conv's
            z1 = (conv1(y).float() * g1).sum()
        (z1 + z2).backward()
        torch.cuda.synchronize()
        res[early] = {"dx": x.grad.float().cpu(), "dgamma": bn.weight.grad.float().cpu(),
                      "dbeta": bn.bias.grad.float().cpu(), "issued": bn_mod.EARLY_ISSUED[0] - issued,
                      "no_early": bool(getattr(bn, "_rtseg_no_early", False))}
    torch.save(res, os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_syncbn_early_reduction_rejected_at_two_consumer_site(tmp_path):
    port = _port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_run, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(180)
    for p in ps:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(2)]
    dx_ref, dg_ref, db_ref = _reference(_data())
    rel = lambda a, b: float((a.double() - b).norm() / b.norm())  # noqa: E731
    for r, rr in enumerate(res):
        on, off = rr[True], rr[False]
        # the early all-reduce was issued from the conv's backward, then rejected: the gradient
        # the BN node received was not the conv's dx alone
        assert on["issued"] == 1 and on["no_early"], on
        assert off["issued"] == 0
        for k in ("dx", "dgamma", "dbeta"):
            torch.testing.assert_close(on[k], off[k], rtol=0, atol=0, msg=f"rank {r} {k}")
        assert rel(on["dx"], dx_ref[r * N:(r + 1) * N]) < 2e-2, r
    # parameter gradients are each rank's contribution (DDP averages them): the sum is the global one
    assert rel(res[0][True]["dgamma"] + res[1][True]["dgamma"], dg_ref) < 2e-2
    assert rel(res[0][True]["dbeta"] + res[1][True]["dbeta"], db_ref) < 2e-2
