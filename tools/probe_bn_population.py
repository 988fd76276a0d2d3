"""Calibrate the zoo train-BN test (tests/test_zoo.py ``check_zoo_hip_matches_torch_path``).

For every zoo model at the GPU test's shape (batch 2, 128 x 256): each BatchNorm's per-channel
population N*H*W; with every BN below a threshold frozen (running statistics), the CPU fp32 gradient
error against CPU fp64 for one batch-statistics step, plus ``draws`` more fp32 errors of
ulp-perturbed models (independent rounding draws, ``test_zoo.perturb_ulp``) -- the spread of the
rounding-noise envelope the HIP path is scored against.
Usage: python tools/probe_bn_population.py [T1,T2,...] [draws] [model,...]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

import test_zoo as tz  # noqa: E402


def main():
    ths = [int(t) for t in (sys.argv[1] if len(sys.argv) > 1 else "0,64,256,1024").split(",")]
    draws = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    keys = sys.argv[3].split(",") if len(sys.argv) > 3 else tz.KEYS
    torch.manual_seed(0)
    x = torch.randn(2, 3, *tz.HW)
    labels = torch.randint(0, 19, (2, *tz.HW))
    for key in keys:
        pops = tz.bn_populations(tz._model(key), x)
        row = [f"{key:12s} minpop {min(pops.values()) if pops else -1:6d}"]
        for t in ths:
            nf = sum(p < t for p in pops.values())
            e = tz.cpu_fp32_vs_fp64_train_bn(key, x, labels, t, draws)
            if draws:
                row.append(f"T={t} ({nf} frozen): plain {e[0]:.2e} draws {min(e[1:]):.2e}..{max(e[1:]):.2e}"
                           f" max/min {max(e) / max(min(e), 1e-30):.1f}")
            else:
                row.append(f"T={t}: {e:.2e} ({nf} frozen)")
        print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
