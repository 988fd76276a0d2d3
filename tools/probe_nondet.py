"""Find the first module whose forward output differs between two identical runs."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
from realtime_semantic_segmentation_pytorch_amd.models import get_model

key, mode = sys.argv[1], sys.argv[2]  # mode: cl | nchw
os.environ["RTSEG_DISABLE_HIP"] = sys.argv[3] if len(sys.argv) > 3 else "1"
c = BaseConfig()
c.model, c.num_class, c.use_aux, c.use_detail_head = key, 19, False, False
torch.manual_seed(0)
fmt = torch.channels_last if mode == "cl" else torch.contiguous_format
m = get_model(c).cuda().to(memory_format=fmt).eval()
x = torch.randn(2, 3, 128, 256, device="cuda").contiguous(memory_format=fmt)
records = []
for name, mod in m.named_modules():
    if len(list(mod.children())) == 0:
        mod.register_forward_hook(lambda mod, i, o, name=name: records.append(
            (name, type(mod).__name__, o.detach().clone() if torch.is_tensor(o) else None,
             [t.detach().clone() for t in i if torch.is_tensor(t)])))
with torch.no_grad():
    m(x)
    first = records
    records = []
    m(x)
    second = records
for (n, t, a, ia), (_, _, b, ib) in zip(first, second):
    if a is None:
        continue
    same_in = all(torch.equal(p, q) for p, q in zip(ia, ib))
    if not torch.equal(a, b):
        print(f"DIFF at {n} ({t}) inputs_equal={same_in} maxdiff={(a - b).abs().max().item():.3e} "
              f"shape={tuple(a.shape)} stride={a.stride()} in_shapes={[tuple(p.shape) for p in ia]} "
              f"in_strides={[p.stride() for p in ia]}", flush=True)
        if same_in:
            break
print("done", flush=True)
