"""Which path's conv weight gradients are accurate?  Recompute every Conv2d weight
gradient in fp64 on the CPU from the recorded input / grad_output and compare
with the GPU result of the HIP path and of the torch path."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import copy

import torch
import torch.nn as nn

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
from realtime_semantic_segmentation_pytorch_amd.core.loss import SegCELoss
from realtime_semantic_segmentation_pytorch_amd.models import get_model


def rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


def run(m, x, labels, disable):
    os.environ["RTSEG_DISABLE_HIP"] = "1" if disable else "0"
    inputs, gouts = {}, {}
    hooks = []
    for name, mod in m.named_modules():
        if type(mod) is nn.Conv2d:
            hooks.append(mod.register_forward_hook(
                lambda mod, i, o, name=name: inputs.__setitem__(name, i[0].detach().clone())))
            hooks.append(mod.register_full_backward_hook(
                lambda mod, gi, go, name=name: gouts.__setitem__(name, go[0].detach().clone())))
    torch.manual_seed(123)
    with ops.defer_final_upsample():
        out = m(x, is_training=True)
    out = out[0] if isinstance(out, (tuple, list)) else out
    SegCELoss(ops.MODE_MEAN)(out, labels).backward()
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    os.environ["RTSEG_DISABLE_HIP"] = "0"
    return m, inputs, gouts


key = sys.argv[1]
c = BaseConfig()
c.model, c.num_class, c.use_aux, c.use_detail_head = key, 19, False, False
torch.manual_seed(0)
base = get_model(c).cuda().to(memory_format=torch.channels_last).train()
x = torch.randn(2, 3, 128, 256, device="cuda").contiguous(memory_format=torch.channels_last)
labels = torch.randint(0, 19, (2, 128, 256), device="cuda")
mh, ih, gh = run(copy.deepcopy(base), x, labels, False)
mt, it, gt = run(copy.deepcopy(base), x, labels, True)
mods_h = dict(mh.named_modules())
mods_t = dict(mt.named_modules())
for name in ih:
    if name not in gh:
        continue
    mod = mods_h[name]
    ref_h = torch.nn.grad.conv2d_weight(ih[name].cpu().double(), mod.weight.shape, gh[name].cpu().double(),
                                        mod.stride, mod.padding, mod.dilation, mod.groups)
    ref_t = torch.nn.grad.conv2d_weight(it[name].cpu().double(), mod.weight.shape, gt[name].cpu().double(),
                                        mod.stride, mod.padding, mod.dilation, mod.groups)
    eh = rel(mods_h[name].weight.grad.cpu(), ref_h)
    et = rel(mods_t[name].weight.grad.cpu(), ref_t)
    flag = " <<<" if max(eh, et) > 1e-4 else ""
    print(f"{name:40s} hip_vs_fp64 {eh:.2e} torch_vs_fp64 {et:.2e} k={tuple(mod.kernel_size)} "
          f"g={mod.groups} go_stride_h={gh[name].stride()} go_stride_t={gt[name].stride()}{flag}", flush=True)
