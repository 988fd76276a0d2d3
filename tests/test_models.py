"""Model-zoo construction, parameter counts, output shapes, checkpoint key ABI (CPU)."""
import pytest
import torch

from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
from realtime_semantic_segmentation_pytorch_amd.models import get_model
from realtime_semantic_segmentation_pytorch_amd.models.ddrnet import DDRNet


def _cfg(**kw):
    c = BaseConfig()
    c.num_class = 19
    for k, v in kw.items():
        setattr(c, k, v)
    return c


@pytest.mark.parametrize("arch,params,keys", [("DDRNet-23-slim", 5.619040, 306),
                                              ("DDRNet-23", 21.990848, 306),
                                              ("DDRNet-39", 33.904576, 474)])
def test_ddrnet_params_keys(arch, params, keys):
    m = get_model(_cfg(model="ddrnet", arch_type=arch, use_aux=True))
    assert isinstance(m, DDRNet)
    n = sum(p.numel() for p in m.parameters()) / 1e6
    assert abs(n - params) < 1e-5
    sd = m.state_dict()
    assert len(sd) == keys
    assert next(iter(sd)) == "conv1.0.weight"
    assert list(sd)[-1] == "aux_head.1.weight"


def test_ddrnet_shapes():
    m = get_model(_cfg(model="ddrnet", use_aux=True)).eval()
    x = torch.randn(2, 3, 128, 256)
    y = m(x)
    assert y.shape == (2, 19, 128, 256)
    m.train()
    y, aux = m(x, is_training=True)
    assert y.shape == (2, 19, 128, 256) and aux[0].shape == (2, 19, 16, 32)
