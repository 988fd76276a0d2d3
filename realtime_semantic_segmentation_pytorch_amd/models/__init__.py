"""Model registry (parity: reference models/__init__.py:47-122).

``get_model(config)`` builds any of the 36 zoo architectures or an SMP-style
encoder/decoder (``config.model='smp'``); ``get_teacher_model`` builds the
knowledge-distillation teacher.  Unlike the reference, family variants are
selectable from the config (``arch_type`` for DDRNet / ESPNet / Lite-HRNet,
``encoder_type`` for STDC / PP-LiteSeg, ``backbone_type`` for ResNet-based
models) -- SURVEY A.1 #9.  Imports are lazy so a model's module is only
loaded when it is requested.
"""
from __future__ import annotations

import importlib
import os

import torch

# key -> (module, class)
MODEL_HUB = {
    "adscnet": ("adscnet", "ADSCNet"), "aglnet": ("aglnet", "AGLNet"),
    "bisenetv1": ("bisenetv1", "BiSeNetv1"), "bisenetv2": ("bisenetv2", "BiSeNetv2"),
    "canet": ("canet", "CANet"), "cfpnet": ("cfpnet", "CFPNet"), "cgnet": ("cgnet", "CGNet"),
    "contextnet": ("contextnet", "ContextNet"), "dabnet": ("dabnet", "DABNet"),
    "ddrnet": ("ddrnet", "DDRNet"), "dfanet": ("dfanet", "DFANet"), "edanet": ("edanet", "EDANet"),
    "enet": ("enet", "ENet"), "erfnet": ("erfnet", "ERFNet"), "esnet": ("esnet", "ESNet"),
    "espnet": ("espnet", "ESPNet"), "espnetv2": ("espnetv2", "ESPNetv2"),
    "farseenet": ("farseenet", "FarSeeNet"), "fastscnn": ("fastscnn", "FastSCNN"),
    "fddwnet": ("fddwnet", "FDDWNet"), "fpenet": ("fpenet", "FPENet"), "fssnet": ("fssnet", "FSSNet"),
    "icnet": ("icnet", "ICNet"), "lednet": ("lednet", "LEDNet"), "linknet": ("linknet", "LinkNet"),
    "lite_hrnet": ("lite_hrnet", "LiteHRNet"), "liteseg": ("liteseg", "LiteSeg"),
    "mininet": ("mininet", "MiniNet"), "mininetv2": ("mininetv2", "MiniNetv2"),
    "ppliteseg": ("pp_liteseg", "PPLiteSeg"), "regseg": ("regseg", "RegSeg"),
    "segnet": ("segnet", "SegNet"), "shelfnet": ("shelfnet", "ShelfNet"), "sqnet": ("sqnet", "SQNet"),
    "stdc": ("stdc", "STDC"), "swiftnet": ("swiftnet", "SwiftNet"),
}

AUX_MODELS = ("bisenetv2", "ddrnet", "icnet")
DETAIL_HEAD_MODELS = ("stdc",)
# which ctor keyword each variant knob maps to, per model
_VARIANT_KW = {
    "arch_type": {"ddrnet": "arch_type", "espnet": "arch_type", "lite_hrnet": "arch_type"},
    "encoder_type": {"stdc": "encoder_type", "ppliteseg": "encoder_type"},
    "backbone_type": {"bisenetv1": "backbone_type", "farseenet": "backbone_type",
                      "linknet": "backbone_type", "shelfnet": "backbone_type",
                      "swiftnet": "backbone_type", "canet": "backbone_type",
                      "liteseg": "backbone_type", "icnet": "backbone_type"},
}


def model_class(key: str):
    if key not in MODEL_HUB:
        raise NotImplementedError(f"Unsupport model type: {key}")
    mod, cls = MODEL_HUB[key]
    return getattr(importlib.import_module(f".{mod}", __name__), cls)


def _variant_kwargs(config, key):
    kw = {}
    for knob, table in _VARIANT_KW.items():
        val = getattr(config, knob, None)
        if val is not None and key in table:
            kw[table[key]] = val
    return kw


def get_model(config):
    """Build the configured model; every BatchNorm2d, depth-wise conv and pooling
    module is routed through the HIP kernels (``ops.convert_batchnorm`` /
    ``ops.convert_depthwise`` / ``ops.convert_pooling``; module classes only --
    parameters and checkpoint keys are unchanged), every other spatial conv drops the
    taps that only read padding at the current input size (``ops.convert_pruned_convs``), and
    plain dense bias-free convs join the autotuned MFMA conv family (``ops.convert_routed_convs``)."""
    from .. import ops

    model = ops.convert_batchnorm(_build_model(config))
    if getattr(config, "hip_depthwise", True):
        ops.convert_depthwise(model)
    if getattr(config, "hip_pooling", True):
        ops.convert_pooling(model)
    if getattr(config, "tap_convs", True):
        ops.convert_tap_convs(model)
    if getattr(config, "dilated_group_convs", True):
        ops.convert_dilated_group_convs(model)
    if getattr(config, "hip_deconv", True):
        ops.convert_transposed_convs(model)
    ops.convert_pruned_convs(model)  # last: every remaining plain spatial conv
    if getattr(config, "routed_convs", True) and os.environ.get("RTSEG_ROUTED_CONVS", "1") != "0":
        ops.convert_routed_convs(model)  # plain dense bias-free convs -> the MFMA conv family
    if getattr(config, "hip_activations", True):
        ops.convert_activations(model)
    ops.convert_pixel_shuffle(model)
    return model


def _build_model(config):
    key = config.model
    if key == "smp":
        from .smp import build_smp_model

        return build_smp_model(config.decoder, config.encoder, getattr(config, "encoder_weights", None),
                               config.num_class)
    cls = model_class(key)
    kw = _variant_kwargs(config, key)
    if key in AUX_MODELS:
        return cls(num_class=config.num_class, use_aux=config.use_aux, **kw)
    if key in DETAIL_HEAD_MODELS:
        return cls(num_class=config.num_class, use_detail_head=config.use_detail_head,
                   use_aux=config.use_aux, **kw)
    if config.use_aux:
        raise ValueError(f"Model {key} does not support auxiliary heads.\n")
    if config.use_detail_head:
        raise ValueError(f"Model {key} does not support detail heads.\n")
    return cls(num_class=config.num_class, **kw)


def get_teacher_model(config, device):
    """SMP teacher loaded from ``config.teacher_ckpt`` (``{'state_dict': ...}``), eval mode."""
    if not config.kd_training:
        return None
    from .smp import DECODER_HUB, build_smp_model

    if config.teacher_decoder not in DECODER_HUB:
        raise ValueError(f"Unsupported teacher decoder type: {config.teacher_decoder}")
    from .. import ops

    model = ops.convert_pruned_convs(ops.convert_pooling(ops.convert_depthwise(ops.convert_batchnorm(
        build_smp_model(config.teacher_decoder, config.teacher_encoder, None, config.num_class)))))
    ckpt_path = config.teacher_ckpt
    if ckpt_path:
        if not os.path.isfile(ckpt_path):
            raise ValueError(f"Could not find teacher checkpoint at path {ckpt_path}.")
        ckpt = torch.load(ckpt_path, map_location="cpu", weights_only=True)
        model.load_state_dict(ckpt["state_dict"])
        del ckpt
    elif not getattr(config, "teacher_random_init", False):
        raise ValueError("kd_training requires config.teacher_ckpt (or teacher_random_init=True)")
    model = model.to(device)
    model.eval()
    for p in model.parameters():
        p.requires_grad_(False)
    return model


def __getattr__(name):  # lazy access to model classes, e.g. models.DDRNet
    for key, (mod, cls) in MODEL_HUB.items():
        if cls == name:
            return model_class(key)
    if name == "LaplacianConv":
        from .stdc import LaplacianConv

        return LaplacianConv
    raise AttributeError(name)
