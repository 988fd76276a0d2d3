"""Where does the fp32 training-gradient error of a zoo model come from?  For each model: CPU
fp32, GPU torch path (NCHW and channels-last) and GPU HIP path (channels-last), each against a
CPU fp64 run of the same step, with train-mode and with frozen BatchNorm.
python tools/probe_zoo_gpu_err.py bisenetv2 stdc ..."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_zoo import HW, _model  # noqa: E402

from realtime_semantic_segmentation_pytorch_amd import ops  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.core.loss import SegCELoss  # noqa: E402


def step(m, x, y):
    m.zero_grad(set_to_none=True)
    with ops.defer_final_upsample():
        out = m(x, is_training=True)
    out = out[0] if isinstance(out, (tuple, list)) else out
    loss = SegCELoss(ops.MODE_MEAN)(out, y)
    loss.backward()
    return torch.cat([p.grad.flatten().double().cpu() for p in m.parameters() if p.grad is not None])


def main():
    for key in sys.argv[1:]:
        for frozen in (False, True):
            torch.manual_seed(0)
            m = _model(key).train()
            for mod in m.modules():
                if isinstance(mod, torch.nn.modules.dropout._DropoutNd):
                    mod.p = 0.0
                if frozen and isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
                    mod.eval()
            g = torch.Generator().manual_seed(1)
            x = torch.randn(2, 3, *HW, generator=g)
            y = torch.randint(0, 19, (2, *HW), generator=g)
            ref = step(copy.deepcopy(m).double(), x.double(), y)
            err = lambda a: ((a - ref).norm() / ref.norm()).item()  # noqa: E731
            row = {"cpu32": err(step(copy.deepcopy(m), x, y))}
            os.environ["RTSEG_DISABLE_HIP"] = "1"
            row["torch_nchw"] = err(step(copy.deepcopy(m).cuda(), x.cuda(), y.cuda()))
            cl = lambda t: t.cuda().contiguous(memory_format=torch.channels_last)  # noqa: E731
            row["torch_cl"] = err(step(copy.deepcopy(m).cuda().to(memory_format=torch.channels_last), cl(x), y.cuda()))
            os.environ.pop("RTSEG_DISABLE_HIP")
            row["hip_cl"] = err(step(copy.deepcopy(m).cuda().to(memory_format=torch.channels_last), cl(x), y.cuda()))
            print(key, "frozen-BN" if frozen else "train-BN", " ".join(f"{k} {v:.2e}" for k, v in row.items()),
                  flush=True)


if __name__ == "__main__":
    main()
