"""Collectives per training step of the DDP + SyncBN path, counted on 2 ranks (gloo, sharing the
GPU; RCCL needs one GPU per rank).

Per step, for DDRNet-23-slim + aux head (reference wiring utils/parallel.py:34-43):
* exactly ONE forward SyncBN all-reduce ([2C+1] fp64 sums) and ONE backward all-reduce ([2C])
  per SyncBatchNorm layer, all on the SyncBN process group (parallel/ddp.py:syncbn_group); the
  forward ones asynchronous (issued from the producing conv's statistics slab, waited at the BN
  finalize) at >= 80 % of the sites;
* the backward ones mostly issued early, asynchronously, from the consumer conv's backward
  (ops.bn.syncbn_bwd_early) -- counted, and required to be > 0.  A site whose output turns out to
  have a second consumer wastes its early reduction once (step 1) and never issues early again;

* DDP gradient buckets: every gradient element reduced exactly once per step, in a fixed number
  of buckets no larger than the configured cap allows (counted through a DDP comm hook).
"""
import math
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SIZE, BS, STEPS, BUCKET_MB = (128, 256), 2, 4, 1


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(rank, world, port, out):
    for k in ("RTSEG_DISABLE_HIP", "RTSEG_CONV_MFMA"):
        os.environ.pop(k, None)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world), RTSEG_DIST_BACKEND="gloo")
    import torch.distributed as dist
    from torch.distributed.algorithms.ddp_comm_hooks import default_hooks

    from realtime_semantic_segmentation_pytorch_amd import ops
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer
    from realtime_semantic_segmentation_pytorch_amd.datasets.synthetic import _masks_like
    from realtime_semantic_segmentation_pytorch_amd.ops import bn as bn_mod
    from realtime_semantic_segmentation_pytorch_amd.parallel.ddp import de_parallel, syncbn_group

    assert ops.load()
    c = BaseConfig()
    c.dataset, c.num_class, c.model, c.arch_type, c.use_aux = "cityscapes", 19, "ddrnet", "DDRNet-23-slim", True
    c.synthetic_data, c.synthetic_len, c.synthetic_size = True, 8, SIZE
    c.crop_size, c.crop_h, c.crop_w = SIZE[0], SIZE[0], SIZE[1]
    c.train_bs, c.val_bs, c.total_epoch = BS, BS, 4
    c.amp_training, c.amp_dtype, c.channels_last = True, "bf16", True
    c.base_workers, c.use_tb, c.save_ckpt, c.load_ckpt, c.use_ema = 0, False, False, False, True
    c.loss_type, c.ddp_bucket_mb = "ohem", BUCKET_MB
    c.save_dir = os.path.join(out, f"save_{rank}")
    c.init_dependent_config()
    tr = SegTrainer(c)
    tr.parallel_model(c)
    ddp = tr.model
    buckets = []

    def hook(state, bucket):
        buckets.append(bucket.buffer().numel())
        return default_hooks.allreduce_hook(None, bucket)

    ddp.register_comm_hook(None, hook)
    sbn = syncbn_group()
    calls = []
    real = dist.all_reduce

    def counting(t, *a, **kw):
        group = kw.get("group", a[1] if len(a) > 1 else None)
        calls.append(("sbn" if group is sbn else "other", t.numel() % 2, bool(kw.get("async_op", False))))
        return real(t, *a, **kw)

    dist.all_reduce = counting
    g = torch.Generator().manual_seed(rank)
    per_step = []
    for _ in range(STEPS):
        calls.clear()
        buckets.clear()
        e0 = bn_mod.EARLY_ISSUED[0]
        img = torch.randn(BS, 3, *SIZE, generator=g)
        msk = _masks_like(g, BS, SIZE[0], SIZE[1], 19, 255, "cpu")
        imgs, masks = tr._prep(img, msk)
        tr.train_step(imgs, masks)
        torch.cuda.synchronize()
        per_step.append({"fwd": sum(1 for k, odd, _ in calls if k == "sbn" and odd == 1),
                         "fwd_async": sum(1 for k, odd, asy in calls if k == "sbn" and odd == 1 and asy),
                         "bwd": sum(1 for k, odd, _ in calls if k == "sbn" and odd == 0),
                         "other": sum(1 for k, _, _ in calls if k != "sbn"),
                         "early": bn_mod.EARLY_ISSUED[0] - e0,
                         "buckets": len(buckets), "bucket_numel": sum(buckets)})
    dist.all_reduce = real
    model = de_parallel(ddp)
    n_sbn = sum(isinstance(m, torch.nn.SyncBatchNorm) for m in model.modules())
    n_grad = sum(p.numel() for p in model.parameters() if p.requires_grad)
    grad_bytes = sum(p.numel() * 4 for p in model.parameters() if p.requires_grad)
    torch.save({"per_step": per_step, "n_sbn": n_sbn, "n_grad": n_grad, "grad_bytes": grad_bytes},
               os.path.join(out, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_syncbn_and_ddp_collectives_per_step(tmp_path):
    port = _port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_run, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(240)
    for p in ps:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(2)]
    assert res[0]["per_step"] == res[1]["per_step"]  # ranks issue the same collectives
    r = res[0]
    print(r)
    cap = BUCKET_MB * 2 ** 20
    for i, st in enumerate(r["per_step"]):
        assert st["fwd"] == r["n_sbn"], st
        # forward statistics all-reduces are issued asynchronously (waited at the BN finalize)
        assert st["fwd_async"] >= 0.8 * st["fwd"], st
        assert st["early"] > 0, st
        assert st["bucket_numel"] == r["n_grad"], st  # every gradient element exactly once
        # the DDP allreduce hook's own dist.all_reduce calls (one per bucket): nothing else
        # all-reduces through Python in a train step
        assert st["other"] == st["buckets"], st
        if i >= 1:  # after step 1's waste (see docstring): one backward all-reduce per layer
            assert st["bwd"] == r["n_sbn"], st
    # DDP rebuilds its buckets from the observed gradient order after the first iterations;
    # from then on a fixed count within what the cap allows
    late = r["per_step"][-2:]
    assert late[0]["buckets"] == late[1]["buckets"] <= math.ceil(r["grad_bytes"] / cap) + 2, late
