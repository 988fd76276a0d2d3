#!/usr/bin/env python3
"""Which parameters carry a zoo model's train-BN gradient error?  Re-runs the exact step of
``tests/test_zoo.py::check_zoo_hip_matches_torch_path`` (batch 2, 128 x 256, batch-statistics BN)
in fp64 on the CPU, CPU fp32, the HIP path (channels-last) and the stock GPU path (NCHW), and
prints, per path, the parameters with the largest share of the squared gradient error.

  python tools/probe_param_err.py ddrnet [bisenetv2 ...]
"""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_zoo as Z  # noqa: E402


class _MP:  # monkeypatch stand-in for Z._run_gpu
    def setenv(self, k, v):
        os.environ[k] = v

    def delenv(self, k, raising=True):
        os.environ.pop(k, None)


def main():
    if os.environ.get("PROBE_NO_TF32") == "1":  # true-fp32 MIOpen / hipBLASLt (no reduced-precision fp32 solvers)
        torch.backends.cudnn.allow_tf32 = False
        torch.backends.cuda.matmul.allow_tf32 = False
    print(f"cudnn.allow_tf32={torch.backends.cudnn.allow_tf32} matmul.allow_tf32={torch.backends.cuda.matmul.allow_tf32}")
    mp = _MP()
    for key in sys.argv[1:]:
        torch.manual_seed(0)
        cpu = Z._model(key)
        for mod in cpu.modules():
            if isinstance(mod, torch.nn.modules.dropout._DropoutNd):
                mod.p = 0.0
        nb = int(os.environ.get("PROBE_BATCH", "2"))
        x = torch.randn(nb, 3, *Z.HW)
        labels = torch.randint(0, 19, (nb, *Z.HW))
        base = copy.deepcopy(cpu).cuda().to(memory_format=torch.channels_last)
        xg = x.cuda().contiguous(memory_format=torch.channels_last)
        y_r, l_r, g_r = Z._run_gpu(copy.deepcopy(cpu).train().double(), x.double(), labels, False, mp)
        y_c, l_c, g_c = Z._run_gpu(copy.deepcopy(cpu).train(), x, labels, False, mp)
        y_h, l_h, g_h = Z._run_gpu(copy.deepcopy(base).train(), xg, labels.cuda(), False, mp)
        y_t, l_t, g_t = Z._run_gpu(copy.deepcopy(cpu).cuda().train(), x.cuda(), labels.cuda(), True, mp)
        ref_sq = sum(g_r[n].double().norm().item() ** 2 for n in g_r)
        flat = lambda g: torch.cat([g[n].double().cpu().flatten() for n in g_r])  # noqa: E731
        fr = flat(g_r)
        for tag, g, y, l in (("cpu fp32", g_c, y_c, l_c), ("HIP", g_h, y_h, l_h), ("stock GPU", g_t, y_t, l_t)):
            fg = flat(g)
            scale = (fg @ fr / (fr @ fr)).item()
            resid = ((fg - scale * fr).norm() / fr.norm()).item()
            yerr = ((y.double().cpu() - y_r.double()).norm() / y_r.double().norm()).item()
            print(f"== {key} {tag}: loss {l.item():.8f} vs fp64 {l_r.item():.8f}; output err {yerr:.2e}; "
                  f"grad = {scale:.6f} x fp64 + residual {resid:.2e}")
            errs = {n: (g[n].double().cpu() - g_r[n].double()).norm().item() ** 2 for n in g_r}
            tot = sum(errs.values())
            print(f"== {key} {tag}: rel grad err {(tot / ref_sq) ** 0.5:.3e}")
            for n, e in sorted(errs.items(), key=lambda kv: -kv[1])[:8]:
                rel = e ** 0.5 / (g_r[n].double().norm().item() + 1e-30)
                print(f"   {e / max(tot, 1e-300):6.1%}  rel {rel:.2e}  |g| {g_r[n].double().norm().item():.2e}  {n}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
