"""Gradient agreement of one DDRNet-23 (+aux) training step against an fp32 stock-PyTorch
reference: stock bf16, HIP bf16 (all rtseg kernels incl. MFMA convs) and HIP fp32 (rtseg BN /
loss / interp kernels, convs on MIOpen).  At random init the BN-heavy backward amplifies
rounding noise layer by layer (two identical stock bf16 runs already differ), so the yardstick
for the bf16 path is the stock bf16 path's own distance to fp32.  Prints per-parameter cosine
similarity to the fp32 reference in model order and a summary."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.datasets import DeviceBatches  # noqa: E402

VARIANTS = [("stock_fp32", False, {"RTSEG_DISABLE_HIP": "1"}), ("stock_bf16", True, {"RTSEG_DISABLE_HIP": "1"}),
            ("hip_bf16", True, {"RTSEG_CONV_MFMA": "1"}), ("hip_fp32", False, {})]


def grads(tr, imgs, masks, amp):
    tr.config.amp_training = amp
    tr.model.zero_grad(set_to_none=True)
    loss, _, _ = tr.compute_loss(imgs, masks)
    loss.backward()
    return float(loss.detach()), {n: p.grad.detach().float().clone() for n, p in tr.model.named_parameters()
                                  if p.grad is not None}


def run(model="ddrnet", arch="DDRNet-23", size=(256, 512)):
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        os.environ.pop(k, None)
    c = BaseConfig()
    c.dataset, c.num_class, c.model, c.arch_type, c.use_aux = "cityscapes", 19, model, arch, True
    c.synthetic_data, c.synthetic_len, c.synthetic_size = True, 8, size
    c.crop_size, c.crop_h, c.crop_w = size[0], size[0], size[1]
    c.train_bs, c.val_bs, c.total_epoch = 4, 4, 2
    c.amp_training, c.amp_dtype, c.channels_last = True, "bf16", True
    c.base_workers, c.use_tb, c.save_ckpt, c.load_ckpt = 0, False, False, False
    c.save_dir = "/tmp/probe_num"
    c.init_dependent_config()
    tr = SegTrainer(c)
    tr.model.train()
    imgs, masks = DeviceBatches(4, size, 19, 255, device=tr.device, pool=1, channels_last=True, seed=0).next()
    res = {}
    for name, amp, env in VARIANTS:
        for k in ("RTSEG_DISABLE_HIP", "RTSEG_CONV_MFMA"):
            os.environ.pop(k, None)
        os.environ.update(env)
        res[name] = grads(tr, imgs, masks, amp)
    for k in ("RTSEG_DISABLE_HIP", "RTSEG_CONV_MFMA"):
        os.environ.pop(k, None)
    ref = res["stock_fp32"][1]
    cos = {v: {n: float(torch.nn.functional.cosine_similarity(g.flatten(), ref[n].flatten(), dim=0))
               for n, g in res[v][1].items() if ref[n].norm() > 1e-8} for v, _, _ in VARIANTS[1:]}
    losses = {v: res[v][0] for v, _, _ in VARIANTS}
    return cos, losses


def main():
    cos, losses = run()
    print("losses:", losses)
    names = list(cos["hip_bf16"])
    print("param".ljust(48) + "".join(v.rjust(12) for v in cos))
    for n in names:
        print(n.ljust(48) + "".join(f"{cos[v][n]:12.5f}" for v in cos))
    for v in cos:
        vals = sorted(cos[v].values())
        print(f"{v}: min {vals[0]:.5f} median {vals[len(vals) // 2]:.5f} mean {sum(vals) / len(vals):.5f}")


if __name__ == "__main__":
    main()
