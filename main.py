#!/usr/bin/env python3
"""Training / prediction entry point (parity: reference main.py:8-21).

  python main.py [--flags]                                  # one GPU (or CPU)
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 main.py [--flags]   # DDP over RCCL

Without torchrun, a training run that sees several GPUs (or ``--spawn_procs N``) starts one
worker process per device itself and trains as single-node DDP over RCCL -- the MI355X
replacement of the reference's single-process ``nn.DataParallel`` mode (reference
utils/parallel.py:7-31); ``--spawn_procs 1`` keeps one device.

Like the reference, the configuration is ``MyConfig`` (``is_testing=True`` by
default -> prediction); unlike the reference, CLI flags are always applied on
top of it (``configs/parser.py``; the reference ships that overlay commented out).
``--no_cli`` ignores the command line entirely.
"""
import os
import sys
import warnings

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from realtime_semantic_segmentation_pytorch_amd.configs import MyConfig, load_parser  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.core import SegTrainer  # noqa: E402

warnings.filterwarnings("ignore")


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawned(local_rank, world, port, argv):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(local_rank),
                      LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world))
    main(argv)


def _spawn_count(config):
    """Worker processes for a run started without a launcher (0: run in this process)."""
    if os.getenv("LOCAL_RANK") is not None or config.is_testing:
        return 0
    n = getattr(config, "spawn_procs", None)
    if n is None:
        import torch

        # device_count() does not initialise the GPU in this process (children own the devices)
        n = torch.cuda.device_count() if getattr(config, "device", None) != "cpu" else 1
    return int(n) if int(n) > 1 else 0


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    config = MyConfig()
    if "--no_cli" in argv:
        argv.remove("--no_cli")
    else:
        config = load_parser(config, argv)
    config.init_dependent_config()
    world = _spawn_count(config)
    if world:
        import torch.multiprocessing as mp

        mp.spawn(_spawned, args=(world, _free_port(), argv), nprocs=world, join=True)
        return None
    trainer = SegTrainer(config)
    if config.is_testing:
        trainer.predict(config)
    else:
        trainer.run(config)
    return trainer


if __name__ == "__main__":
    main()
