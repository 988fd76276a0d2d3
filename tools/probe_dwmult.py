"""Probe: depth-wise conv with channel multiplier (DFANet XceptionBlock) through MIOpen, pure torch."""
import sys
import torch

fmt = torch.channels_last if sys.argv[1] == "cl" else torch.contiguous_format
dtype = torch.float32 if sys.argv[2] == "f32" else torch.bfloat16
for cin, mult, stride, hw in [(12, 4, 2, (64, 128)), (24, 4, 2, (32, 64)), (48, 4, 2, (16, 32))]:
    conv = torch.nn.Conv2d(cin, cin * mult, 3, stride, 1, groups=cin, bias=False).cuda().to(dtype)
    conv = conv.to(memory_format=fmt)
    x = torch.randn(2, cin, *hw, device="cuda", dtype=dtype).contiguous(memory_format=fmt).requires_grad_()
    y = conv(x)
    y.float().square().sum().backward()
    torch.cuda.synchronize()
    print("ok", sys.argv[1:], cin, mult, stride, hw, flush=True)
