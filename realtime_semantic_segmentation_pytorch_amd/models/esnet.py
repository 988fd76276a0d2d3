"""ESNet (arXiv:1906.09826) -- efficient symmetric network of factorized conv units.

Parity target: reference models/esnet.py (ESNet :16-52, build_blocks :55-66,
FCU :69-90 -- (K,1)/(1,K) factorized pairs + residual; PFCU :93-138 -- three
parallel dilated factorized branches summed with the residual).
"""
from __future__ import annotations

import torch.nn as nn

from .enet import InitialBlock as DownsamplingUnit
from .modules import Activation, ConvBNAct, DeConvBNAct


class ESNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, act_type="relu"):
        super().__init__()
        self.block1_down = DownsamplingUnit(n_channel, 16, act_type)
        self.block1 = build_blocks("fcu", 16, 3, K=3, act_type=act_type)
        self.block2_down = DownsamplingUnit(16, 64, act_type)
        self.block2 = build_blocks("fcu", 64, 2, K=5, act_type=act_type)
        self.block3_down = DownsamplingUnit(64, 128, act_type)
        self.block3 = build_blocks("pfcu", 128, 3, r1=2, r2=5, r3=9, act_type=act_type)
        self.block4_up = DeConvBNAct(128, 64, act_type=act_type)
        self.block4 = build_blocks("fcu", 64, 2, K=5, act_type=act_type)
        self.block5_up = DeConvBNAct(64, 16, act_type=act_type)
        self.block5 = build_blocks("fcu", 16, 2, K=3, act_type=act_type)
        self.full_conv = DeConvBNAct(16, num_class, act_type=act_type)

    def forward(self, x, is_training=False):
        for name in ("block1_down", "block1", "block2_down", "block2", "block3_down", "block3",
                     "block4_up", "block4", "block5_up", "block5", "full_conv"):
            x = getattr(self, name)(x)
        return x


def build_blocks(block_type, channels, num_block, K=None, r1=None, r2=None, r3=None, act_type="relu"):
    if block_type == "fcu":
        make = lambda: FCU(channels, K, act_type)  # noqa: E731
    elif block_type == "pfcu":
        make = lambda: PFCU(channels, r1, r2, r3, act_type)  # noqa: E731
    else:
        raise NotImplementedError(f"Unsupported block type: {block_type}.\n")
    return nn.Sequential(*[make() for _ in range(num_block)])


def _factorized(channels, k, dilation, act_type, last_act):
    """conv(k,1) -> act -> ConvBNAct(1,k); children 0 / 1 / 2."""
    return [nn.Conv2d(channels, channels, (k, 1), padding=((k - 1) // 2 * dilation, 0), dilation=dilation,
                      bias=False),
            Activation(act_type, inplace=True),
            ConvBNAct(channels, channels, (1, k), dilation=dilation, act_type=last_act,
                      **({"inplace": True} if last_act != "none" else {}))]


class FCU(nn.Module):
    def __init__(self, channels, K, act_type):
        super().__init__()
        if K is None:
            raise AssertionError("K should not be None.\n")
        self.conv = nn.Sequential(*_factorized(channels, K, 1, act_type, act_type),
                                  *_factorized(channels, K, 1, act_type, "none"))
        self.act = Activation(act_type)

    def forward(self, x):
        h = x
        for m in list(self.conv)[:5]:
            h = m(h)
        # BN + residual + act fused in one pass
        return self.conv[5](h, residual=x, act=self.act)


class PFCU(nn.Module):
    def __init__(self, channels, r1, r2, r3, act_type):
        super().__init__()
        if r1 is None or r2 is None or r3 is None:
            raise AssertionError
        self.conv0 = nn.Sequential(*_factorized(channels, 3, 1, act_type, act_type))
        self.conv_left = nn.Sequential(*_factorized(channels, 3, r1, act_type, "none"))
        self.conv_mid = nn.Sequential(*_factorized(channels, 3, r2, act_type, "none"))
        self.conv_right = nn.Sequential(*_factorized(channels, 3, r3, act_type, "none"))
        self.act = Activation(act_type)

    def forward(self, x):
        h = self.conv0(x)
        acc = self.conv_left(h) + self.conv_mid(h) + x
        r = self.conv_right[1](self.conv_right[0](h))
        return self.conv_right[2](r, residual=acc, act=self.act)
