"""Graph-captured training step (SegTrainer.graph_step): forward + loss + backward replayed from
one HIP graph must train like the eager step (reference core/seg_trainer.py:38-119 step)."""
import torch


def _trainer(tmp_path, graph, model="ddrnet"):
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer

    c = BaseConfig()
    c.dataset, c.num_class, c.model = "cityscapes", 19, model
    if model == "ddrnet":
        c.arch_type, c.use_aux = "DDRNet-23-slim", True
    c.loss_type, c.optimizer_type = "ohem", "sgd"
    c.synthetic_data, c.synthetic_len, c.crop_size = True, 8, 256
    c.train_bs = c.val_bs = 4
    c.base_workers, c.use_tb, c.save_ckpt, c.load_ckpt = 0, False, False, False
    c.save_dir = str(tmp_path / ("g" if graph else "e"))
    c.use_ema = True
    c.graph_step, c.graph_warmup = graph, 2
    c.random_seed = 1
    c.init_dependent_config()
    return SegTrainer(c)


def test_graph_step_trains_like_eager(tmp_path, model):
    torch.manual_seed(0)
    xs = [torch.randn(4, 3, 256, 512, device="cuda").contiguous(memory_format=torch.channels_last) for _ in range(6)]
    ys = [torch.randint(0, 19, (4, 256, 512), device="cuda") for _ in range(6)]
    out = {}
    for graph in (False, True):
        torch.manual_seed(1)
        tr = _trainer(tmp_path, graph, model)
        if model == "enet":  # dropout RNG streams differ between eager and replay: compare without it
            for m in tr.model.modules():
                if isinstance(m, torch.nn.modules.dropout._DropoutNd):
                    m.p = 0.0
        losses = [float(tr.train_step(x, y)[0]) for x, y in zip(xs, ys)]
        out[graph] = (losses, {k: v.detach().float().clone() for k, v in tr.model.state_dict().items()},
                      {n for n, p in tr.model.named_parameters() if p.grad is None})
        if graph:
            assert tr._gstep["graph"] is not None  # steps 3.. replayed the captured graph
    le, lg = out[False][0], out[True][0]
    for a, b in zip(le, lg):
        assert abs(a - b) <= 2e-2 * abs(a) + 1e-3, (le, lg)
    se, sg = out[False][1], out[True][1]
    num = sum(float((se[k] - sg[k]).norm() ** 2) for k in se if se[k].is_floating_point())
    den = sum(float(se[k].norm() ** 2) for k in se if se[k].is_floating_point())
    assert (num / den) ** 0.5 < 1e-2
    # parameters without a gradient stay without one under graph capture (no persistent zero
    # gradient that weight decay / momentum would then act on)
    assert out[False][2] == out[True][2], (out[False][2] ^ out[True][2])


if __name__ == "__main__":  # run in a child process by tests/test_isolated_gpu.py
    import pathlib
    import sys
    import tempfile

    sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[2]))
    with tempfile.TemporaryDirectory() as d:
        for model in ("ddrnet", "enet"):
            test_graph_step_trains_like_eager(pathlib.Path(d), model)
            print(f"graph step {model}: ok", flush=True)
