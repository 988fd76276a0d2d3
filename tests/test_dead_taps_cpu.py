"""No stock-path conv ever sees a padding-only tap.

The round-4 driver GPU suite aborted in ``test_zoo.py``'s stock-bf16 yardstick run
(``RTSEG_DISABLE_HIP=1``): in that mode the depth-wise, grouped-dilated and tap-conv modules fell
back to ``F.conv2d`` / ``nn.Conv2d.forward`` WITHOUT dead-tap pruning, so LEDNet's / FDDWNet's /
DABNet's dilated depth-wise convs (dilation up to 17 on 8..32-row maps at 128 x 256) reached
MIOpen with taps that read nothing but zero padding -- the geometry class behind the round-2/3
faults (``ops/dilated.py`` header, ``profiles/r3_fault``).  Every fallback now goes through
``pruned_conv2d``; this test pins it for the whole zoo: with the HIP dispatch forced off, no
``torch.nn.functional.conv2d`` call of a forward + backward at 128 x 256 receives a
``has_dead_taps`` geometry.  (On CPU the modules take the same fallback branches as under
``RTSEG_DISABLE_HIP=1`` on the GPU.)
"""
import pytest
import torch
import torch.nn.functional as F

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
from realtime_semantic_segmentation_pytorch_amd.models import AUX_MODELS, MODEL_HUB, get_model
from realtime_semantic_segmentation_pytorch_amd.ops.dilated import has_dead_taps

HW = (128, 256)


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def _recording_conv2d(real, bad):
    def conv2d(input, weight, bias=None, stride=1, padding=0, dilation=1, groups=1):
        if not isinstance(padding, str) and input.dim() == 4:
            geom = (tuple(input.shape[2:]), tuple(weight.shape[2:]), _pair(stride), _pair(padding), _pair(dilation))
            if has_dead_taps(*geom):
                bad.append(geom)
        return real(input, weight, bias, stride, padding, dilation, groups)

    return conv2d


def _model(key):
    c = BaseConfig()
    c.model, c.num_class = key, 19
    c.use_aux = key in AUX_MODELS
    c.use_detail_head = False
    torch.manual_seed(0)
    return get_model(c)


@pytest.mark.parametrize("key", sorted(MODEL_HUB))
def test_stock_fallback_never_sees_dead_taps_cpu(key, monkeypatch):
    monkeypatch.setenv("RTSEG_DISABLE_HIP", "1")
    bad = []
    monkeypatch.setattr(F, "conv2d", _recording_conv2d(F.conv2d, bad))
    m = _model(key).train()
    x = torch.randn(2, 3, *HW)
    out = m(x, is_training=True) if key in AUX_MODELS else m(x)
    main = out[0] if isinstance(out, (tuple, list)) else out
    main.float().square().mean().backward()
    m.eval()
    with torch.no_grad():
        m(x[:1])
    assert not bad, f"{key}: {len(bad)} conv calls with padding-only taps, e.g. {bad[:3]}"


def test_recorder_catches_an_unpruned_dead_tap_cpu(monkeypatch):
    """The recorder itself: a raw dilation-17 (3, 1) conv on a 16-row map is flagged; the same
    conv through ``pruned_conv2d`` is not and gives the same output."""
    bad = []
    real = F.conv2d
    monkeypatch.setattr(F, "conv2d", _recording_conv2d(real, bad))
    x, w = torch.randn(1, 4, 16, 32), torch.randn(4, 4, 3, 1)
    y = F.conv2d(x, w, None, 1, (17, 0), (17, 1))
    assert len(bad) == 1
    bad.clear()
    torch.testing.assert_close(ops.pruned_conv2d(x, w, None, (1, 1), (17, 0), (17, 1), 1), y)
    assert not bad
