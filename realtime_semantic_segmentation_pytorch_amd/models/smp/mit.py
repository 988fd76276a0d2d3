"""Mix Transformer (SegFormer's MiT-B0..B5) encoders for the SMP-style decoders.

Parity target: the ``mit_b*`` encoders that the reference reaches through
segmentation_models_pytorch (reference models/__init__.py:67-81: ``mit_b*`` with PAN is built at
encoder output stride 32, and ``deeplabv3`` / ``deeplabv3p`` / ``linknet`` / ``unetpp`` are rejected).
SMP is not installed here, so parity with its module tree is by construction and its outputs
are "parity unpinned" (tests/test_smp.py checks shapes, the key layout and the SMP contract).

Module / state_dict layout follows SMP's ``MixVisionTransformerEncoder``:
``patch_embed{1..4}.{proj,norm}``, ``block{1..4}.<i>.{norm1,attn.{q,kv,proj,sr,norm},norm2,
mlp.{fc1,dwconv.dwconv,fc2}}``, ``norm{1..4}`` and the unused ImageNet ``head``.  ``forward``
returns ``[x, empty(B, 0, H/2, W/2), f4, f8, f16, f32]`` -- the zero-channel stride-2 feature
is SMP's placeholder for the stage MiT does not have.

MI355X notes: attention runs through ``F.scaled_dot_product_attention`` (the fused ROCm flash
kernels); the spatial-reduction conv and the Mix-FFN depth-wise conv are channels-last convs.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

# name: (embed_dims, depths); every variant: heads (1, 2, 5, 8), sr (8, 4, 2, 1), mlp ratio 4
MIT_SPECS = {
    "mit_b0": ((32, 64, 160, 256), (2, 2, 2, 2)),
    "mit_b1": ((64, 128, 320, 512), (2, 2, 2, 2)),
    "mit_b2": ((64, 128, 320, 512), (3, 4, 6, 3)),
    "mit_b3": ((64, 128, 320, 512), (3, 4, 18, 3)),
    "mit_b4": ((64, 128, 320, 512), (3, 8, 27, 3)),
    "mit_b5": ((64, 128, 320, 512), (3, 6, 40, 3)),
}
_HEADS = (1, 2, 5, 8)
_SR = (8, 4, 2, 1)


def _drop_path(x, p, training):
    if p == 0.0 or not training:
        return x
    keep = 1.0 - p
    mask = x.new_empty((x.shape[0],) + (1,) * (x.dim() - 1)).bernoulli_(keep)
    return x * mask / keep


class DropPath(nn.Module):
    def __init__(self, p=0.0):
        super().__init__()
        self.p = p

    def forward(self, x):
        return _drop_path(x, self.p, self.training)


class DWConv(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dwconv = nn.Conv2d(dim, dim, 3, 1, 1, bias=True, groups=dim)

    def forward(self, x, h, w):
        b, n, c = x.shape
        x = x.transpose(1, 2).reshape(b, c, h, w)
        return self.dwconv(x).flatten(2).transpose(1, 2)


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.dwconv = DWConv(hidden)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x, h, w):
        return self.fc2(self.act(self.dwconv(self.fc1(x), h, w)))


class Attention(nn.Module):
    """Efficient self-attention: keys / values from a sr x sr strided-conv reduced sequence."""

    def __init__(self, dim, num_heads, sr_ratio):
        super().__init__()
        assert dim % num_heads == 0
        self.num_heads = num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.q = nn.Linear(dim, dim, bias=True)
        self.kv = nn.Linear(dim, dim * 2, bias=True)
        self.proj = nn.Linear(dim, dim)
        self.sr_ratio = sr_ratio
        if sr_ratio > 1:
            self.sr = nn.Conv2d(dim, dim, sr_ratio, sr_ratio)
            self.norm = nn.LayerNorm(dim)

    def forward(self, x, h, w):
        b, n, c = x.shape
        nh = self.num_heads
        q = self.q(x).reshape(b, n, nh, c // nh).transpose(1, 2)
        if self.sr_ratio > 1:
            xs = self.sr(x.transpose(1, 2).reshape(b, c, h, w)).flatten(2).transpose(1, 2)
            xs = self.norm(xs)
        else:
            xs = x
        kv = self.kv(xs).reshape(b, -1, 2, nh, c // nh).permute(2, 0, 3, 1, 4)
        out = F.scaled_dot_product_attention(q, kv[0], kv[1], scale=self.scale)
        return self.proj(out.transpose(1, 2).reshape(b, n, c))


class Block(nn.Module):
    def __init__(self, dim, num_heads, sr_ratio, drop_path):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, num_heads, sr_ratio)
        self.drop_path = DropPath(drop_path)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, dim * 4)

    def forward(self, x, h, w):
        x = x + self.drop_path(self.attn(self.norm1(x), h, w))
        return x + self.drop_path(self.mlp(self.norm2(x), h, w))


class OverlapPatchEmbed(nn.Module):
    def __init__(self, patch_size, stride, in_chans, embed_dim):
        super().__init__()
        self.proj = nn.Conv2d(in_chans, embed_dim, patch_size, stride, patch_size // 2)
        self.norm = nn.LayerNorm(embed_dim)

    def forward(self, x):
        x = self.proj(x)
        h, w = x.shape[2:]
        return self.norm(x.flatten(2).transpose(1, 2)), h, w


class MixVisionTransformerEncoder(nn.Module):
    def __init__(self, name="mit_b0", depth=5, drop_path_rate=0.1):
        super().__init__()
        if name not in MIT_SPECS:
            raise ValueError(f"Unknown Mix Transformer `{name}`")
        dims, depths = MIT_SPECS[name]
        self._depth = depth
        self.out_channels = (3, 0) + tuple(dims)
        self.out_channels = self.out_channels[: depth + 1]
        self.output_stride = 32
        rates = torch.linspace(0, drop_path_rate, sum(depths)).tolist()
        cur = 0
        in_ch = 3
        for i in range(4):
            ps, st = (7, 4) if i == 0 else (3, 2)
            setattr(self, f"patch_embed{i + 1}", OverlapPatchEmbed(ps, st, in_ch, dims[i]))
            setattr(self, f"block{i + 1}", nn.ModuleList(
                [Block(dims[i], _HEADS[i], _SR[i], rates[cur + j]) for j in range(depths[i])]))
            setattr(self, f"norm{i + 1}", nn.LayerNorm(dims[i], eps=1e-6))
            cur += depths[i]
            in_ch = dims[i]
        self.head = nn.Linear(dims[3], 1000)  # ImageNet classifier of the checkpoint layout; unused
        self.apply(_init_weights)

    def make_dilated(self, output_stride):
        if output_stride != 32:
            raise ValueError("MixVisionTransformer encoder does not support dilated mode")

    def forward_features(self, x):
        b = x.shape[0]
        outs = []
        for i in range(1, 5):
            x, h, w = getattr(self, f"patch_embed{i}")(x)
            for blk in getattr(self, f"block{i}"):
                x = blk(x, h, w)
            x = getattr(self, f"norm{i}")(x)
            x = x.reshape(b, h, w, -1).permute(0, 3, 1, 2).contiguous()
            outs.append(x)
        return outs

    def forward(self, x):
        b, _, h, w = x.shape
        dummy = torch.empty([b, 0, h // 2, w // 2], dtype=x.dtype, device=x.device)
        return [x, dummy] + self.forward_features(x)[: self._depth - 1]

    def load_state_dict(self, state_dict, strict=True):
        """An ImageNet checkpoint's classifier (``head.*``) is optional, as in SMP."""
        sd = {k: v for k, v in state_dict.items() if not k.startswith("head.")}
        res = super().load_state_dict(sd, strict=False)
        missing = [k for k in res.missing_keys if not k.startswith("head.")]
        if strict and (missing or res.unexpected_keys):
            raise RuntimeError(f"MiT state_dict mismatch: missing {missing[:6]}, unexpected {res.unexpected_keys[:6]}")
        return res


def _init_weights(m):
    if isinstance(m, nn.Linear):
        nn.init.trunc_normal_(m.weight, std=0.02)
        if m.bias is not None:
            nn.init.zeros_(m.bias)
    elif isinstance(m, nn.LayerNorm):
        nn.init.ones_(m.weight)
        nn.init.zeros_(m.bias)
    elif isinstance(m, nn.Conv2d):
        fan_out = m.kernel_size[0] * m.kernel_size[1] * m.out_channels // m.groups
        m.weight.data.normal_(0, math.sqrt(2.0 / fan_out))
        if m.bias is not None:
            m.bias.data.zero_()
