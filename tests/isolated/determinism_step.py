"""One process: DDRNet-23-slim (+ aux head, OHEM) trained for 3 ``SegTrainer.train_step`` calls
with ``config.deterministic``; prints one JSON line with the SHA-256 of every parameter, buffer
and EMA tensor (bytes) and the loss bits.  tests/test_determinism_gpu.py runs it twice and
compares (bit-reproducibility across processes)."""
import hashlib
import json
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

SIZE, BS, STEPS = (256, 512), 2, 3


def main():
    from realtime_semantic_segmentation_pytorch_amd import ops
    from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
    from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer
    from realtime_semantic_segmentation_pytorch_amd.datasets.synthetic import _masks_like
    from realtime_semantic_segmentation_pytorch_amd.parallel import de_parallel

    assert ops.load()
    c = BaseConfig()
    c.dataset, c.num_class = "cityscapes", 19
    c.model, c.arch_type, c.use_aux = "ddrnet", "DDRNet-23-slim", True
    c.synthetic_data, c.synthetic_len, c.synthetic_size = True, 8, SIZE
    c.crop_size, c.crop_h, c.crop_w = SIZE[0], SIZE[0], SIZE[1]
    c.train_bs, c.val_bs, c.total_epoch = BS, BS, 4
    c.amp_training, c.amp_dtype, c.channels_last = True, "bf16", True
    c.base_workers, c.use_tb, c.save_ckpt, c.load_ckpt, c.use_ema = 0, False, False, False, True
    c.deterministic = True
    c.save_dir = os.environ.get("DET_OUT", "/tmp/det_step")
    c.init_dependent_config()
    tr = SegTrainer(c)
    tr.parallel_model(c)
    g = torch.Generator().manual_seed(11)
    losses = []
    for _ in range(STEPS):
        img = torch.randn(BS, 3, *SIZE, generator=g)
        msk = _masks_like(g, BS, SIZE[0], SIZE[1], 19, 255, "cpu")
        imgs, masks = tr._prep(img, msk)
        loss, _ = tr.train_step(imgs, masks)
        losses.append(struct.pack("<f", float(loss)).hex())
    torch.cuda.synchronize()
    model = de_parallel(tr.model)
    h = hashlib.sha256()
    tensors = list(model.state_dict().items()) + [("ema." + k, v) for k, v in tr.ema_model.ema.state_dict().items()]
    for name, t in tensors:
        h.update(name.encode())
        h.update(t.detach().reshape(-1).contiguous().cpu().view(torch.uint8).numpy().tobytes() if t.numel() else b"")
    print(json.dumps({"sha256": h.hexdigest(), "losses": losses, "n_tensors": len(tensors)}), flush=True)


if __name__ == "__main__":
    main()
