"""KD teacher as a captured HIP graph (SegTrainer._teacher_forward) == the eager teacher.
Reference: core/seg_trainer.py:94-101 (teacher forward under no_grad, KD loss)."""
import torch


def _trainer(tmp_path, graph):
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer

    c = BaseConfig()
    c.dataset, c.num_class, c.model, c.arch_type = "cityscapes", 19, "ddrnet", "DDRNet-23-slim"
    c.use_aux = False
    c.kd_training, c.teacher_model, c.teacher_encoder, c.teacher_decoder = True, "smp", "resnet18", "deeplabv3p"
    c.teacher_random_init = True
    c.synthetic_data, c.synthetic_len, c.crop_size = True, 4, 128
    c.train_bs = c.val_bs = 2
    c.base_workers, c.use_tb, c.save_ckpt = 0, False, False
    c.save_dir = str(tmp_path)
    c.kd_teacher_graph = graph
    c.init_dependent_config()
    return SegTrainer(c)


def test_graph_teacher_matches_eager(tmp_path):
    torch.manual_seed(0)
    tr = _trainer(tmp_path, True)
    x = torch.randn(2, 3, 128, 256, device="cuda").contiguous(memory_format=torch.channels_last)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        eager = tr.teacher_model(x).float()
        g1 = tr._teacher_forward(x).float().clone()
        g2 = tr._teacher_forward(x * 0.5).float().clone()  # replay with new data
        eager2 = tr.teacher_model(x * 0.5).float()
    assert tr._teacher_engine[1].graph is not None
    for a, b in ((g1, eager), (g2, eager2)):
        rel = ((a - b).norm() / b.norm()).item()
        assert rel < 2e-2, rel
    y = torch.randint(0, 19, (2, 128, 256), device="cuda")
    loss, _, extras = tr.compute_loss(x, y)
    loss.backward()
    assert torch.isfinite(loss) and torch.isfinite(extras["loss_kd"])


if __name__ == "__main__":  # run in a child process by tests/test_isolated_gpu.py
    import pathlib
    import sys
    import tempfile

    sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[2]))
    with tempfile.TemporaryDirectory() as d:
        test_graph_teacher_matches_eager(pathlib.Path(d))
        print("kd teacher graph: ok", flush=True)
