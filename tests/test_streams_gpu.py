"""Concurrent branches in inference (ops/streams.py): DDRNet's low- and high-resolution branches
on two HIP streams give the same bits as one stream, eagerly and replayed from a captured HIP graph
(utils/inference.py), and the aux head is no longer evaluated when it is not returned.

MIOpen runs with ``cudnn.deterministic`` here: without it its solvers differ run to run in the last
bf16 bit even on one stream (measured: 2.4e-4 between two single-stream runs), which would hide
what this checks -- that the fork / join orders every read after its write."""
import pytest
import torch

from realtime_semantic_segmentation_pytorch_amd import ops

pytestmark = pytest.mark.gpu


def _model(arch="DDRNet-23-slim"):
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.models import get_model

    torch.manual_seed(0)
    c = BaseConfig()
    c.model, c.arch_type, c.num_class, c.use_aux = "ddrnet", arch, 19, True
    m = get_model(c).cuda().eval()
    with torch.no_grad():  # non-trivial running statistics
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.uniform_(-0.1, 0.1)
                mod.running_var.uniform_(0.5, 1.5)
    return m.to(memory_format=torch.channels_last)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_ddrnet_branch_streams_bitwise(monkeypatch, dtype):
    from realtime_semantic_segmentation_pytorch_amd.ops import streams

    assert ops.load()
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    m = _model()
    x = torch.randn(1, 3, 256, 512, device="cuda").contiguous(memory_format=torch.channels_last)
    out = {}
    for on in (False, True, False, True):  # interleaved: decisions cached by the first pass
        monkeypatch.setattr(streams, "_ON", on)
        before = streams.FORKS[0]
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
            y = m(x)
        torch.cuda.synchronize()
        assert (streams.FORKS[0] > before) == on
        out.setdefault(on, []).append(y.float().clone())
    assert torch.equal(out[True][1], out[False][1])
    assert torch.equal(out[True][0], out[True][1])


def test_ddrnet_branch_streams_in_graph(monkeypatch):
    from realtime_semantic_segmentation_pytorch_amd.ops import streams
    from realtime_semantic_segmentation_pytorch_amd.utils.inference import InferenceEngine

    assert ops.load()
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    monkeypatch.setattr(streams, "_ON", True)
    m = _model("DDRNet-23")
    x = torch.randn(1, 3, 512, 1024, device="cuda")
    before = streams.FORKS[0]
    eng = InferenceEngine(m, (1, 3, 512, 1024), dtype=torch.bfloat16, warmup=2)
    assert streams.FORKS[0] > before  # the captured forward forked
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        ref = m(x.contiguous(memory_format=torch.channels_last)).float()
    got = eng(x).float()
    got2 = eng(x).float()
    torch.cuda.synchronize()
    assert torch.equal(got, got2)
    assert torch.equal(got, ref)


def test_aux_head_skipped_in_inference():
    m = _model()
    calls = []
    m.aux_head.register_forward_hook(lambda *a: calls.append(1))
    x = torch.randn(1, 3, 128, 256, device="cuda")
    with torch.no_grad():
        m(x)
    assert not calls
    m.train()
    y, (aux,) = m(torch.randn(2, 3, 128, 256, device="cuda"), is_training=True)
    assert calls and aux.shape[1] == 19
