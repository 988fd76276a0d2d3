"""HIP SyncBatchNorm (ops/bn.py + bn_act.hip, RCCL/gloo all-reduce of fp64 sums) across 2 ranks
vs single-process BatchNorm2d over the concatenated batch: forward output, input / weight /
bias gradients, running statistics and num_batches_tracked -- for the plain BN, the fused
BN + residual + ReLU tail, and the conv-epilogue statistics path (conv_igemm slab ->
bn_slab_sums -> all-reduce).  Reference wiring: utils/parallel.py:34-43 (SyncBN + DDP).

Two processes share the one GPU of the box and talk over gloo (RCCL needs one GPU per rank)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, C, H, W = 4, 64, 12, 20


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, C, H, W, generator=g) * 2 + 0.5
    res = torch.randn(N, C, H, W, generator=g)
    gy = torch.randn(N, C, H, W, generator=g)
    conv_w = torch.randn(C, C, 3, 3, generator=g) / (9 * C) ** 0.5
    bn_w = torch.rand(C, generator=g) + 0.5
    bn_b = torch.randn(C, generator=g) * 0.1
    return x, res, gy, conv_w, bn_w, bn_b


def _make_bn(bn_w, bn_b, sync, pg=None):
    import torch.nn as nn

    from realtime_semantic_segmentation_pytorch_amd.ops import convert_batchnorm

    bn = nn.BatchNorm2d(C)
    with torch.no_grad():
        bn.weight.copy_(bn_w)
        bn.bias.copy_(bn_b)
    if sync:
        bn = nn.SyncBatchNorm.convert_sync_batchnorm(bn, process_group=pg)
    convert_batchnorm(bn)
    return bn.cuda()


def _case(kind, x, res, gy, conv_w, bn, conv=None):
    """-> (y, dx, dres)"""
    from realtime_semantic_segmentation_pytorch_amd import ops

    x = x.cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    r = res.cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    g = gy.cuda().contiguous(memory_format=torch.channels_last)
    if kind == "plain":
        y = bn(x)
    elif kind == "tail":
        y = ops.bn_act(x, bn, "relu", residual=r)
    else:  # conv with the BN statistics in its epilogue, bf16
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = ops.conv_bn_act(x.to(torch.bfloat16), conv, bn, "relu")
    y.float().backward(g)
    return y.detach().float(), x.grad.float(), (r.grad.float() if r.grad is not None else None)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      RTSEG_CONV_MFMA="1")
    import torch.distributed as dist
    import torch.nn as nn

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pg = dist.new_group(ranks=list(range(world)))
    x, res, gy, conv_w, bn_w, bn_b = _data()
    sl = slice(rank * N // world, (rank + 1) * N // world)
    res_out = {}
    for kind in ("plain", "tail", "conv"):
        bn = _make_bn(bn_w, bn_b, True, pg)
        conv = None
        if kind == "conv":
            conv = nn.Conv2d(C, C, 3, 1, 1, bias=False).cuda()
            with torch.no_grad():
                conv.weight.copy_(conv_w)
            conv = conv.to(memory_format=torch.channels_last)
        y, dx, dres = _case(kind, x[sl], res[sl], gy[sl], conv_w, bn, conv)
        dw, db = bn.weight.grad.clone(), bn.bias.grad.clone()
        dist.all_reduce(dw)  # DDP would sum (then average) the per-rank contributions
        dist.all_reduce(db)
        res_out[kind] = dict(y=y.cpu(), dx=dx.cpu(), dres=None if dres is None else dres.cpu(), dw=dw.cpu(),
                             db=db.cpu(), rm=bn.running_mean.cpu(), rv=bn.running_var.cpu(),
                             nbt=bn.num_batches_tracked.cpu(),
                             cw=None if conv is None else conv.weight.grad.clone().cpu())
        if conv is not None:
            cw = res_out[kind]["cw"].cuda()
            dist.all_reduce(cw)
            res_out[kind]["cw"] = cw.cpu()
    torch.save(res_out, os.path.join(out, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_hip_syncbn_two_ranks_matches_full_batch_bn(tmp_path):
    import torch.nn as nn

    from realtime_semantic_segmentation_pytorch_amd import ops

    assert ops.load(), "HIP extension must load on the GPU box"
    mp.spawn(_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    got = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in (0, 1)]
    x, res, gy, conv_w, bn_w, bn_b = _data()
    os.environ["RTSEG_CONV_MFMA"] = "1"
    try:
        for kind in ("plain", "tail", "conv"):
            bn = _make_bn(bn_w, bn_b, False)
            conv = None
            if kind == "conv":
                conv = nn.Conv2d(C, C, 3, 1, 1, bias=False).cuda()
                with torch.no_grad():
                    conv.weight.copy_(conv_w)
                conv = conv.to(memory_format=torch.channels_last)
            y, dx, dres = _case(kind, x, res, gy, conv_w, bn, conv)
            tol = dict(rtol=2e-2, atol=3e-2) if kind == "conv" else dict(rtol=1e-4, atol=2e-4)
            y2 = torch.cat([got[0][kind]["y"], got[1][kind]["y"]])
            dx2 = torch.cat([got[0][kind]["dx"], got[1][kind]["dx"]])
            torch.testing.assert_close(y2, y.cpu(), **tol, msg=f"{kind}: forward")
            torch.testing.assert_close(dx2, dx.cpu(), **tol, msg=f"{kind}: grad input")
            if dres is not None:
                torch.testing.assert_close(torch.cat([got[0][kind]["dres"], got[1][kind]["dres"]]), dres.cpu(),
                                           **tol, msg=f"{kind}: grad residual")
            for r in (0, 1):
                g = got[r][kind]
                torch.testing.assert_close(g["dw"], bn.weight.grad.cpu(), rtol=1e-3, atol=5e-2 if kind == "conv" else 1e-3,
                                           msg=f"{kind}: grad weight")
                torch.testing.assert_close(g["db"], bn.bias.grad.cpu(), rtol=1e-3, atol=5e-2 if kind == "conv" else 1e-3,
                                           msg=f"{kind}: grad bias")
                torch.testing.assert_close(g["rm"], bn.running_mean.cpu(), rtol=1e-3, atol=1e-3, msg=f"{kind}: mean")
                torch.testing.assert_close(g["rv"], bn.running_var.cpu(), rtol=2e-3, atol=1e-3, msg=f"{kind}: var")
                assert int(g["nbt"]) == int(bn.num_batches_tracked) == 1
                if conv is not None:
                    torch.testing.assert_close(g["cw"], conv.weight.grad.cpu(), rtol=3e-2, atol=3e-2,
                                               msg="conv weight grad")
    finally:
        os.environ.pop("RTSEG_CONV_MFMA", None)


# ------------------------------------------------------------------ pooled attention / [N,C,1,1] BNs
def _block(kind):
    from realtime_semantic_segmentation_pytorch_amd.models.bisenetv1 import AttentionRefinementModule
    from realtime_semantic_segmentation_pytorch_amd.models.bisenetv2 import ContextEmbeddingBlock

    torch.manual_seed(3)
    return AttentionRefinementModule(C) if kind == "arm" else ContextEmbeddingBlock(C, C)


def _block_run(m, x, gy):
    x = x.cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = m(x)
    y.backward(gy.cuda().contiguous(memory_format=torch.channels_last))
    bns = [b for b in m.modules() if isinstance(b, torch.nn.modules.batchnorm._BatchNorm)]
    return (y.detach().float().cpu(), x.grad.float().cpu(),
            {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None},
            [(b.running_mean.cpu(), b.running_var.cpu()) for b in bns])


def _block_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import torch.nn as nn

    from realtime_semantic_segmentation_pytorch_amd.ops import convert_batchnorm

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pg = dist.new_group(ranks=list(range(world)))
    x, _, gy, *_ = _data()
    sl = slice(rank * N // world, (rank + 1) * N // world)
    res = {}
    for kind in ("arm", "ce"):
        m = nn.SyncBatchNorm.convert_sync_batchnorm(_block(kind), process_group=pg)
        convert_batchnorm(m)
        m = m.cuda().to(memory_format=torch.channels_last).train()
        y, dx, grads, stats = _block_run(m, x[sl], gy[sl])
        for g in grads.values():
            dist.all_reduce(g)
        res[kind] = dict(y=y, dx=dx, grads={k: v.cpu() for k, v in grads.items()}, stats=stats)
    torch.save(res, os.path.join(out, f"blk{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_syncbn_pooled_attention_and_context_embedding_two_ranks():
    """SyncBN in the pooled attention branch (BiSeNetV1 / STDC ARM: pooled_conv_bn_act) and in
    BiSeNetV2's context-embedding BN on [N, C, 1, 1]: 2 ranks x half batch == one process over
    the whole batch (reference utils/parallel.py:36-37 syncs every BN)."""
    import tempfile

    from realtime_semantic_segmentation_pytorch_amd import ops
    from realtime_semantic_segmentation_pytorch_amd.ops import convert_batchnorm

    assert ops.load()
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_block_worker, args=(2, _port(), tmp), nprocs=2, join=True)
        got = [torch.load(os.path.join(tmp, f"blk{r}.pt"), weights_only=True) for r in (0, 1)]
    x, _, gy, *_ = _data()
    for kind in ("arm", "ce"):
        m = _block(kind)
        convert_batchnorm(m)
        m = m.cuda().to(memory_format=torch.channels_last).train()
        y, dx, grads, stats = _block_run(m, x, gy)
        tol = dict(rtol=1e-4, atol=2e-4)
        torch.testing.assert_close(torch.cat([got[0][kind]["y"], got[1][kind]["y"]]), y, **tol, msg=f"{kind}: y")
        torch.testing.assert_close(torch.cat([got[0][kind]["dx"], got[1][kind]["dx"]]), dx, **tol, msg=f"{kind}: dx")
        for r in (0, 1):
            for n, g in grads.items():
                # relative to the tensor's norm: the context-embedding BNs normalise over N = 4
                # pooled values, so single elements carry fp32 summation-order noise.  The pooled
                # BN's bias feeds a 1x1 conv followed by a training-mode BN, which cancels any
                # per-channel constant: its true gradient is 0 and both sides hold only rounding
                # noise, hence the absolute floor.
                a, b = got[r][kind]["grads"][n].double(), g.cpu().double()
                diff, ref = (a - b).norm().item(), b.norm().item()
                assert diff < 2e-3 * ref + 1e-5 * b.numel() ** 0.5, \
                    f"{kind}: grad {n} |diff| {diff:.3e} vs |ref| {ref:.3e}"
            for (rm, rv), (rm2, rv2) in zip(got[r][kind]["stats"], stats):
                torch.testing.assert_close(rm, rm2, rtol=1e-3, atol=1e-4, msg=f"{kind}: running mean")
                torch.testing.assert_close(rv, rv2, rtol=2e-3, atol=1e-4, msg=f"{kind}: running var")


def _pooled_bn_worker(rank, world, port, out, fused):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import torch.nn as nn

    from realtime_semantic_segmentation_pytorch_amd.ops import convert_batchnorm

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pg = dist.new_group(ranks=list(range(world)))
    torch.manual_seed(5)
    bn = nn.BatchNorm2d(C)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    bn = nn.SyncBatchNorm.convert_sync_batchnorm(bn, process_group=pg)
    if fused:
        bn = convert_batchnorm(nn.Sequential(bn))[0]
    bn = bn.cuda().train()
    g = torch.Generator().manual_seed(6)
    x = torch.randn(4, C, 1, 1, generator=g) * 2 + 0.3
    gy = torch.randn(4, C, 1, 1, generator=g)
    sl = slice(rank * 2, rank * 2 + 2)
    xs = x[sl].cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = bn(xs)
    y.backward(gy[sl].cuda().contiguous(memory_format=torch.channels_last))
    gw, gb = bn.weight.grad.clone(), bn.bias.grad.clone()
    dist.all_reduce(gw)
    dist.all_reduce(gb)
    torch.save({"y": y.detach().cpu(), "dx": xs.grad.cpu(), "gw": gw.cpu(), "gb": gb.cpu()},
               os.path.join(out, f"pbn{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fused", [False, True])
def test_syncbn_on_pooled_vectors_two_ranks(fused):
    """SyncBN over [N, C, 1, 1] (BiSeNetV2 context embedding): 2 ranks x 2 vectors == 1 process x
    4 vectors, for torch's SyncBatchNorm (fused=False: the reference semantics) and ours."""
    import tempfile

    import torch.nn as nn

    torch.manual_seed(5)
    bn = nn.BatchNorm2d(C)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    bn = bn.cuda().train()
    g = torch.Generator().manual_seed(6)
    x = (torch.randn(4, C, 1, 1, generator=g) * 2 + 0.3).cuda().requires_grad_(True)
    gy = torch.randn(4, C, 1, 1, generator=g).cuda()
    y = bn(x)
    y.backward(gy)
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_pooled_bn_worker, args=(2, _port(), tmp, fused), nprocs=2, join=True)
        got = [torch.load(os.path.join(tmp, f"pbn{r}.pt"), weights_only=True) for r in (0, 1)]
    torch.testing.assert_close(torch.cat([got[0]["y"], got[1]["y"]]), y.detach().cpu(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(torch.cat([got[0]["dx"], got[1]["dx"]]), x.grad.cpu(), rtol=1e-3, atol=1e-4)
    for r in (0, 1):
        torch.testing.assert_close(got[r]["gw"], bn.weight.grad.cpu(), rtol=1e-3, atol=1e-4, msg="weight grad")
        torch.testing.assert_close(got[r]["gb"], bn.bias.grad.cpu(), rtol=1e-3, atol=1e-4, msg="bias grad")
