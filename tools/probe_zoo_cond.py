"""fp32 vs fp64 training-gradient error of zoo models on the CPU at several (batch, H, W): finds a
size at which the fp32 step is well conditioned (tests/test_zoo.py ZOO_TRAIN_SIZE).
python tools/probe_zoo_cond.py bisenetv2 stdc ..."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_zoo import _model  # noqa: E402

from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.core.loss import SegCELoss  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.ops.interp import DeferredLogits  # noqa: E402


def step(m, x, y):
    with ops.defer_final_upsample():
        out = m(x, is_training=True)
    out = out[0] if isinstance(out, (tuple, list)) else out
    loss = SegCELoss(ops.MODE_MEAN)(out, y)
    loss.backward()
    return torch.cat([p.grad.flatten().double() for p in m.parameters() if p.grad is not None])


def main():
    sizes = [(2, 128, 256), (4, 128, 256), (8, 128, 256), (4, 256, 512), (8, 256, 512)]
    bn_eval = os.environ.get("BN_EVAL") == "1"
    for key in sys.argv[1:]:
        for n, h, w in sizes:
            torch.manual_seed(0)
            m = _model(key).train()
            if bn_eval:  # frozen BatchNorm: the batch-statistics conditioning is out of the picture
                for mod in m.modules():
                    if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
                        mod.eval()
            for mod in m.modules():
                if isinstance(mod, torch.nn.modules.dropout._DropoutNd):
                    mod.p = 0.0
            g = torch.Generator().manual_seed(1)
            x = torch.randn(n, 3, h, w, generator=g)
            y = torch.randint(0, 19, (n, h, w), generator=g)
            g32 = step(copy.deepcopy(m), x, y)
            g64 = step(copy.deepcopy(m).double(), x.double(), y)
            err = ((g32 - g64).norm() / g64.norm()).item()
            print(f"{key} n={n} {h}x{w}: grad err {err:.3e}", flush=True)
            if err < 1e-3:
                break


if __name__ == "__main__":
    main()
