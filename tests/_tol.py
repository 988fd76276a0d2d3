"""Kernel-vs-fp32 tolerances for the conv kernel tests.

The references are fp32 PyTorch convs of the SAME bf16-valued operands, so a correct kernel differs
from them only by (a) the rounding of a bf16 output, at most half a bf16 ulp = 2^-9 |v|, and (b) the
fp32 accumulation order, ~1e-6 of the largest output.  The bounds below allow one full ulp plus
1e-3 x max|ref| where sums cancel near zero -- 20x tighter than the rounds-1-5 bound of
2e-2 x max|ref|.  A dropped 8-channel slice of one tap moves the affected
outputs by ~10 % of their typical size and fails both.
"""
import torch

BF16_RTOL = 2.0 ** -8
BF16_FLOOR = 1e-3
F32_RTOL, F32_FLOOR = 1e-3, 1e-4


def bf16_close(got, ref, floor=BF16_FLOOR):
    """A bf16 kernel output against its fp32 reference."""
    torch.testing.assert_close(got.float(), ref.float(), rtol=BF16_RTOL,
                               atol=floor * ref.abs().max().item() + 1e-6)


def f32_close(got, ref):
    """An fp32 kernel output (weight gradients: split-K partial sums in fp32) against fp32."""
    torch.testing.assert_close(got.float(), ref.float(), rtol=F32_RTOL,
                               atol=F32_FLOOR * ref.abs().max().item() + 1e-6)
