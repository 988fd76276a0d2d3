"""SegNet (arXiv:1511.00561).

Parity target: reference models/segnet.py (SegNet :14-42, DownsampleBlock
:45-59 with max-pool indices, UpsampleBlock :62-80 with max-unpool).  VGG-style
encoder/decoder, full-resolution output.
"""
from __future__ import annotations

import torch.nn as nn

from .modules import ConvBNAct

# (extra conv?) per stage 1..5
_EXTRA = (False, False, True, True, True)


class SegNet(nn.Module):
    def __init__(self, num_class=1, n_channel=3, hid_channel=64, act_type="relu"):
        super().__init__()
        h = hid_channel
        widths = (n_channel, h, 2 * h, 4 * h, 8 * h, 8 * h)
        for i in range(5):
            setattr(self, f"down_stage{i + 1}", DownsampleBlock(widths[i], widths[i + 1], act_type, _EXTRA[i]))
        up_io = {5: (8 * h, 8 * h), 4: (8 * h, 4 * h), 3: (4 * h, 2 * h), 2: (2 * h, h), 1: (h, h)}
        for s in (5, 4, 3, 2, 1):
            setattr(self, f"up_stage{s}", UpsampleBlock(*up_io[s], act_type, _EXTRA[s - 1]))
        self.classifier = ConvBNAct(h, num_class, act_type=act_type)

    def forward(self, x, is_training=False):
        idx = []
        for i in range(1, 6):
            x, ind = getattr(self, f"down_stage{i}")(x)
            idx.append(ind)
        for s in (5, 4, 3, 2, 1):
            x = getattr(self, f"up_stage{s}")(x, idx[s - 1])
        return self.classifier(x)


class DownsampleBlock(nn.Module):
    def __init__(self, in_channels, out_channels, act_type="relu", extra_conv=False):
        super().__init__()
        n = 3 if extra_conv else 2
        self.conv = nn.Sequential(*[ConvBNAct(in_channels if i == 0 else out_channels, out_channels, 3,
                                              act_type=act_type, inplace=True) for i in range(n)])
        self.pool = nn.MaxPool2d(kernel_size=2, stride=2, return_indices=True)

    def forward(self, x):
        return self.pool(self.conv(x))


class UpsampleBlock(nn.Module):
    def __init__(self, in_channels, out_channels, act_type="relu", extra_conv=False):
        super().__init__()
        self.pool = nn.MaxUnpool2d(kernel_size=2, stride=2)
        mid = in_channels if extra_conv else out_channels
        layers = [ConvBNAct(in_channels, in_channels, 3, act_type=act_type, inplace=True),
                  ConvBNAct(in_channels, mid, 3, act_type=act_type, inplace=True)]
        if extra_conv:
            layers.append(ConvBNAct(in_channels, out_channels, 3, act_type=act_type, inplace=True))
        self.conv = nn.Sequential(*layers)

    def forward(self, x, indices):
        return self.conv(self.pool(x, indices))
