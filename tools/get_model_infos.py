"""Model parameters and MACs (parity: reference tools/get_model_infos.py:9-33).

  python tools/get_model_infos.py --model ddrnet [--arch_type DDRNet-23]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from realtime_semantic_segmentation_pytorch_amd.configs import MyConfig, load_parser  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.models import get_model  # noqa: E402
from realtime_semantic_segmentation_pytorch_amd.utils.model_info import count_macs, count_params  # noqa: E402


def cal_model_params(config, imgw=1024, imgh=512):
    model = get_model(config)
    print(f"\nModel: {config.model}\nEncoder: {config.encoder}\nDecoder: {config.decoder}")
    params = count_params(model)
    macs = count_macs(model, (1, 3, imgh, imgw))
    print(f"Number of parameters: {params / 1e6:.2f}M")
    print(f"Computational complexity: {macs / 1e9:.2f} GMac ({imgw}x{imgh})\n")
    return params, macs


if __name__ == "__main__":
    cal_model_params(load_parser(MyConfig(), sys.argv[1:]))
