"""Bisect a 2-rank vs 1-process mismatch of tests/test_ddp_model_gpu.py by kernel family.

For each variant (all HIP kernels, then one family at a time back on its stock formulation via
``RTSEG_HIP_OFF=<family>``) the fp32 2-rank and 1-process runs are repeated and the update
cosine printed, with the parameters of largest RELATIVE update difference (in forward order:
the earliest layer whose update is off is downstream of where the paths diverge).

    python tools/probe_ddp_bisect.py --model stdc2_aux [--families bn,pool,gate,interp,loss]
"""
import argparse
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_ddp_model_gpu as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="stdc2_aux")
    ap.add_argument("--families", default=",bn,pool,gate,interp,loss,act,dw")
    ap.add_argument("--amp", action="store_true")
    a = ap.parse_args()
    init = T._init_params(a.model, None)
    keys = sorted(init)
    for fam in a.families.split(","):
        if fam:
            os.environ["RTSEG_HIP_OFF"] = fam
        else:
            os.environ.pop("RTSEG_HIP_OFF", None)
        with tempfile.TemporaryDirectory() as out:
            T._spawn(1, T._port(), out, a.model, a.amp)
            T._spawn(2, T._port(), out, a.model, a.amp)
            one = torch.load(os.path.join(out, f"{a.model}_{int(a.amp)}_w1_r0.pt"), weights_only=True)
            r0 = torch.load(os.path.join(out, f"{a.model}_{int(a.amp)}_w2_r0.pt"), weights_only=True)
        d1 = T._flat(one["params1"]["params"], keys) - T._flat(init, keys)
        d2 = T._flat(r0["params1"]["params"], keys) - T._flat(init, keys)
        cos = float(torch.dot(d1, d2) / (d1.norm() * d2.norm()))
        rows = []
        for k in keys:
            u1 = (one["params1"]["params"][k] - init[k]).double()
            u2 = (r0["params1"]["params"][k] - init[k]).double()
            if u1.norm() > 1e-3 * d1.norm() / len(keys) ** 0.5:
                rows.append((float((u1 - u2).norm() / u1.norm()), k))
        worst = sorted(rows, reverse=True)[:10]
        print(f"[{fam or 'all-hip'}] update cos {cos:.6f}; losses 1-proc {one['losses']} 2-rank {r0['losses']}")
        order = {k: i for i, k in enumerate(init)}  # named_parameters order = forward-ish order
        for rel, k in sorted(worst, key=lambda t: order[t[1]]):
            print(f"    {rel:8.3f}  {k}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
