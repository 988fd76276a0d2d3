#!/usr/bin/env python3
"""Training / prediction entry point (parity: reference main.py:8-21).

  python main.py [--flags]                                  # one GPU (or CPU)
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 main.py [--flags]   # DDP over RCCL

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


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    config = MyConfig()
    if "--no_cli" in argv:
        argv.remove("--no_cli")
    else:
        config = load_parser(config, argv)
    config.init_dependent_config()
    trainer = SegTrainer(config)
    if config.is_testing:
        trainer.predict(config)
    else:
        trainer.run(config)
    return trainer


if __name__ == "__main__":
    main()
