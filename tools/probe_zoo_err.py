"""Train-step error of the HIP path (all kernels / without the depth-wise kernels) and of the
torch path against a CPU fp64 run, for zoo models (GPU box).  python tools/probe_zoo_err.py dfanet ..."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_zoo import HW, _model, _run_gpu  # noqa: E402


class _MP:
    def setenv(self, k, v):
        os.environ[k] = v

    def delenv(self, k, raising=False):
        os.environ.pop(k, None)


def main():
    mp = _MP()
    for key in sys.argv[1:]:
        torch.manual_seed(0)
        cpu = _model(key)
        for mod in cpu.modules():
            if isinstance(mod, torch.nn.modules.dropout._DropoutNd):
                mod.p = 0.0
        x = torch.randn(2, 3, *HW)
        labels = torch.randint(0, 19, (2, *HW))
        base = copy.deepcopy(cpu).cuda().to(memory_format=torch.channels_last).train()
        xg = x.cuda().contiguous(memory_format=torch.channels_last)
        y_r, l_r, g_r = _run_gpu(copy.deepcopy(cpu).train().double(), x.double(), labels, False, mp)
        cat = lambda g: torch.cat([g[n].flatten().double().cpu() for n in g_r])  # noqa: E731
        err = lambda a, b: ((a.double().cpu() - b.double().cpu()).norm() / (b.double().cpu().norm() + 1e-30)).item()  # noqa: E731
        rows = []
        for name, dis, dw, sep, pool in (("hip", False, "1", "1", "1"), ("hip-no-dw", False, "0", "1", "1"),
                                         ("hip-no-sep", False, "1", "0", "1"), ("hip-no-pool", False, "1", "1", "0"),
                                         ("torch", True, "1", "1", "1")):
            os.environ["RTSEG_DWCONV"] = dw
            os.environ["RTSEG_INTERP_SEP"] = sep
            os.environ["RTSEG_POOL"] = pool
            y, l, g = _run_gpu(copy.deepcopy(base), xg, labels.cuda(), dis, mp)
            rows.append(f"{name}: y {err(y, y_r):.2e} loss {abs(l.item() - l_r.item()):.2e} grad {err(cat(g), cat(g_r)):.2e}")
        os.environ["RTSEG_DWCONV"] = "1"
        print(key, " | ".join(rows), flush=True)


if __name__ == "__main__":
    main()
