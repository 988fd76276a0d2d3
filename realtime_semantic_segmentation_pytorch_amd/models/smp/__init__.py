"""SMP-compatible encoder/decoder models (``config.model='smp'``) and the KD teacher.

Parity: reference models/__init__.py:42-44 (``decoder_hub``), :67-81
(``smp`` branch incl. the ``mit_b*`` special cases) and :102-122 (teacher).
segmentation_models_pytorch is not installed in this environment, so the nine
decoders are native re-implementations with SMP's module layout (see
``base.py``); encoders: ResNet-18/34/50/101/152, ResNeXt-50/101, MobileNetV2, MiT-B0..B5,
VGG-11/13/16/19(+BN), DenseNet-121/161/169/201, EfficientNet-B0..B7, SE-ResNet-50/101/152 and
SE-ResNeXt-50/101 (``encoders_extra.py``).
"""
from __future__ import annotations

from .base import SegmentationHead, SegmentationModel
from .deeplab import DeepLabV3, DeepLabV3Plus
from .encoders import ENCODERS, get_encoder
from .fpn import FPN
from .linknet import Linknet
from .manet import MAnet
from .pan import PAN
from .pspnet import PSPNet
from .unet import Unet, UnetPlusPlus

DECODER_HUB = {"deeplabv3": DeepLabV3, "deeplabv3p": DeepLabV3Plus, "fpn": FPN, "linknet": Linknet,
               "manet": MAnet, "pan": PAN, "pspnet": PSPNet, "unet": Unet, "unetpp": UnetPlusPlus}


def build_smp_model(decoder, encoder, encoder_weights=None, num_class=1, in_channels=3):
    """``decoder_hub[decoder](encoder_name=encoder, encoder_weights=..., in_channels=3, classes=num_class)``."""
    if decoder not in DECODER_HUB:
        raise ValueError(f"Unsupported decoder type: {decoder}")
    encoder = encoder or "resnet18"
    if encoder.startswith("mit_b") and decoder in ("deeplabv3", "deeplabv3p", "linknet", "unetpp"):
        raise ValueError(f"Encoder `{encoder}` is not supported for `{decoder}")
    if encoder.startswith("mit_b") and decoder == "pan":  # reference models/__init__.py:69-73
        return DECODER_HUB[decoder](encoder_name=encoder, encoder_weights=encoder_weights, encoder_output_stride=32,
                                    in_channels=in_channels, classes=num_class)
    return DECODER_HUB[decoder](encoder_name=encoder, encoder_weights=encoder_weights, in_channels=in_channels,
                                classes=num_class)


__all__ = ["DECODER_HUB", "ENCODERS", "build_smp_model", "get_encoder", "SegmentationHead", "SegmentationModel",
           "DeepLabV3", "DeepLabV3Plus", "FPN", "Linknet", "MAnet", "PAN", "PSPNet", "Unet", "UnetPlusPlus"]
