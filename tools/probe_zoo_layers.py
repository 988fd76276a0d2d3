"""Where does a zoo model's HIP fp32 training-step error (tests/test_zoo.py train-BN pass) come
from?  For ``key``, with the small-population BatchNorms frozen as in the test:
* the whole-model gradient / loss error against CPU fp64 with every HIP family on, then with each
  family switched off in turn (``RTSEG_HIP_OFF``) -- the family whose removal closes the gap;
* the forward output of every leaf-level block (ConvBNAct, pools, ...) against fp64, in execution
  order -- the first block whose error jumps.
python tools/probe_zoo_layers.py segnet [families, default bn,pool]
"""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_zoo as Z  # noqa: E402

from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.core.loss import SegCELoss  # noqa: E402


def run(m, x, y, record=None):
    hooks = []
    if record is not None:
        for name, mod in m.named_modules():
            if name and (not list(mod.children()) or type(mod).__name__ in ("ConvBNAct",)):
                def hook(mod_, args, out, name=name):
                    o = out[0] if isinstance(out, (tuple, list)) else out
                    if torch.is_tensor(o) and o.is_floating_point():
                        record.append((name, o.detach().double().cpu()))
                hooks.append(mod.register_forward_hook(hook))
    with ops.defer_final_upsample():
        out = m(x, is_training=True)
    out = out[0] if isinstance(out, (tuple, list)) else out
    loss = SegCELoss(ops.MODE_MEAN)(out, y)
    loss.backward()
    for h in hooks:
        h.remove()
    g = torch.cat([p.grad.flatten().double().cpu() for _, p in m.named_parameters() if p.grad is not None])
    return float(loss), g


def main():
    key = sys.argv[1]
    fams = (sys.argv[2] if len(sys.argv) > 2 else "bn,pool").split(",")
    torch.manual_seed(0)
    cpu = Z._no_dropout(Z._model(key))
    x = torch.randn(2, 3, *Z.HW)
    labels = torch.randint(0, 19, (2, *Z.HW))
    pops = Z.bn_populations(cpu, x)
    prep = lambda m: Z.freeze_small_bn(m.train(), pops)  # noqa: E731
    rec_r, rec_h, rec_n, rec_c = [], [], [], []
    l_r, g_r = run(prep(copy.deepcopy(cpu).double()), x.double(), labels, rec_r)
    xg = x.cuda().contiguous(memory_format=torch.channels_last)
    base = copy.deepcopy(cpu).cuda().to(memory_format=torch.channels_last)
    err = lambda g: float((g - g_r).norm() / g_r.norm())  # noqa: E731
    for off in [""] + fams + ["nocudnn"]:
        torch.backends.cudnn.enabled = off != "nocudnn"  # convs left to PyTorch: native fp32 GEMM convs
        if off == "nocudnn":
            os.environ.pop("RTSEG_HIP_OFF", None)
        elif off == "all":  # the stock PyTorch path on the same channels-last tensors
            os.environ["RTSEG_DISABLE_HIP"] = "1"
        elif off:
            os.environ["RTSEG_HIP_OFF"] = off
        else:
            os.environ.pop("RTSEG_HIP_OFF", None)
        rec = rec_h if not off else (rec_n if off == "nocudnn" else None)
        l_h, g_h = run(prep(copy.deepcopy(base)), xg, labels.cuda(), rec)
        print(f"{key} HIP fp32 (off: {off or '-'}): grad err {err(g_h):.2e} loss err {abs(l_h - l_r):.2e}", flush=True)
    os.environ.pop("RTSEG_HIP_OFF", None)
    os.environ.pop("RTSEG_DISABLE_HIP", None)
    torch.backends.cudnn.enabled = True
    l_c, g_c = run(prep(copy.deepcopy(cpu)), x, labels, rec_c)
    print(f"{key} CPU fp32: grad err {err(g_c):.2e} loss err {abs(l_c - l_r):.2e}")
    ref = {}
    for n, b in rec_r:
        ref.setdefault(n, b)
    fwd = lambda rec: {n: float((a - ref[n]).norm() / (ref[n].norm() + 1e-30)) for n, a in rec  # noqa: E731
                       if n in ref and ref[n].shape == a.shape}
    eh, en, ec = fwd(rec_h), fwd(rec_n), fwd(rec_c)
    print(f"  {'block':40s} fwd err vs fp64: HIP, HIP without MIOpen, CPU fp32")
    for n in eh:
        print(f"  {n:40s} {eh[n]:.2e} {en.get(n, float('nan')):.2e} {ec.get(n, float('nan')):.2e}")

if __name__ == "__main__":
    main()
