"""Command-line overlay for configs (parity: reference configs/parser.py:4-182).

Same flag names and semantics (every default is ``None`` = "keep the config
value"; boolean flags are store_true/store_false toggles like the reference),
with two fixes from SURVEY A.1 #19: values are assigned with ``setattr`` (no
``exec``) and list-valued flags (``--aux_coef``, ``--class_weights``,
``--randscale``) parse comma-separated numbers instead of splitting a string
into characters.
"""
from __future__ import annotations

import argparse

MODEL_CHOICES = [
    "adscnet", "aglnet", "bisenetv1", "bisenetv2", "canet", "cfpnet", "cgnet", "contextnet",
    "dabnet", "ddrnet", "dfanet", "edanet", "enet", "erfnet", "esnet", "espnet", "espnetv2",
    "farseenet", "fastscnn", "fddwnet", "fpenet", "fssnet", "icnet", "lednet", "linknet",
    "lite_hrnet", "liteseg", "mininet", "mininetv2", "ppliteseg", "regseg", "segnet", "shelfnet",
    "sqnet", "stdc", "swiftnet", "smp",
]
DECODER_CHOICES = ["deeplabv3", "deeplabv3p", "fpn", "linknet", "manet", "pan", "pspnet", "unet",
                   "unetpp"]


def float_list(text: str):
    vals = [float(v) for v in str(text).replace("(", "").replace(")", "").replace("[", "")
            .replace("]", "").split(",") if v.strip()]
    return vals[0] if len(vals) == 1 else vals


# (flag, kind, extra) ; kind: str/int/float/list/true/false
_SPEC = [
    # dataset
    ("dataset", str, {"choices": ["cityscapes", "custom"]}), ("dataroot", str, {}),
    ("data_root", str, {}), ("num_class", int, {}), ("ignore_index", int, {}),
    # model
    ("model", str, {"choices": MODEL_CHOICES}), ("encoder", str, {}),
    ("decoder", str, {"choices": DECODER_CHOICES}), ("encoder_weights", str, {}),
    ("arch_type", str, {}), ("encoder_type", str, {}), ("backbone_type", str, {}),
    # detail head
    ("use_detail_head", "true", {}), ("detail_thrs", float, {}), ("detail_loss_coef", float, {}),
    ("dice_loss_coef", float, {}), ("bce_loss_coef", float, {}),
    # training
    ("total_epoch", int, {}), ("base_lr", float, {}), ("train_bs", int, {}),
    ("use_aux", "true", {}), ("no_aux", "true", {"dest": "no_aux"}), ("aux_coef", "list", {}), ("logger_name", str, {}),
    # validating
    ("val_bs", int, {}), ("begin_val_epoch", int, {}), ("val_interval", int, {}),
    # testing
    ("is_testing", "true", {}), ("train", "true", {"dest": "train_mode"}), ("test_bs", int, {}), ("test_data_folder", str, {}),
    ("colormap", str, {"choices": ["cityscapes", "custom"]}), ("save_mask", "false", {}),
    ("blend_prediction", "false", {}), ("blend_alpha", float, {}),
    # loss
    ("loss_type", str, {"choices": ["ce", "ohem"]}), ("class_weights", "list", {}),
    ("ohem_thrs", float, {}), ("reduction", str, {"choices": ["mean", "sum"]}),
    # scheduler / optimizer
    ("lr_policy", str, {"choices": ["cos_warmup", "linear", "step"]}), ("warmup_epochs", int, {}),
    ("step_size", int, {}), ("optimizer_type", str, {"choices": ["sgd", "adam", "adamw"]}),
    ("momentum", float, {}), ("weight_decay", float, {}),
    # monitoring
    ("save_ckpt", "false", {}), ("save_dir", str, {}), ("use_tb", "false", {}),
    ("tb_log_dir", str, {}), ("ckpt_name", str, {}),
    # training setting
    ("amp_training", "true", {}), ("resume_training", "false", {}), ("load_ckpt", "false", {}),
    ("load_ckpt_path", str, {}), ("base_workers", int, {}), ("random_seed", int, {}),
    ("use_ema", "true", {}),
    # augmentation
    ("crop_size", int, {}), ("crop_h", int, {}), ("crop_w", int, {}), ("scale", float, {}),
    ("randscale", "list", {}), ("brightness", float, {}), ("contrast", float, {}),
    ("saturation", float, {}), ("h_flip", float, {}), ("v_flip", float, {}),
    ("train_size", int, {}), ("test_size", int, {}),
    # DDP
    ("synBN", "false", {}), ("local_rank", int, {}), ("local-rank", int, {"dest": "local_rank"}),
    # KD
    ("kd_training", "true", {}), ("teacher_ckpt", str, {}), ("teacher_model", str, {}),
    ("teacher_encoder", str, {}), ("teacher_decoder", str, {"choices": DECODER_CHOICES}),
    ("kd_loss_type", str, {"choices": ["kl_div", "mse"]}), ("kd_loss_coefficient", float, {}),
    ("kd_temperature", float, {}),
    # MI355X knobs
    ("amp_dtype", str, {"choices": ["bf16", "fp16"]}), ("no_channels_last", "true",
                                                        {"dest": "no_channels_last"}),
    ("no_fused_loss", "true", {"dest": "no_fused_loss"}), ("ddp_bucket_mb", int, {}),
    ("gpu_aug", "true", {}), ("spawn_procs", int, {}), ("graph_step", "true", {}), ("synthetic_data", "true", {}), ("synthetic_len", int, {}),
    ("synthetic_learnable", "true", {}), ("synthetic_cell", int, {}), ("max_train_itrs", int, {}),
    ("cudnn_benchmark", "true", {}), ("deterministic", "true", {}),
    ("log_interval", int, {}), ("device", str, {}),
    ("no_fused_optimizer", "true", {"dest": "no_fused_optimizer"}),
]


def get_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X real-time semantic segmentation")
    for name, kind, extra in _SPEC:
        kw = dict(extra)
        kw.setdefault("default", None)
        if kind == "true":
            kw["action"] = "store_true"
        elif kind == "false":
            kw["action"] = "store_false"
        elif kind == "list":
            kw["type"] = float_list
        else:
            kw["type"] = kind
        p.add_argument(f"--{name}", **kw)
    return p


def load_parser(config, argv=None):
    """Overlay every explicitly-given CLI flag onto ``config``.  An unknown or misspelled flag
    is an error (argparse exits with usage), never silently ignored."""
    parser = get_parser()
    args, unknown = parser.parse_known_args(argv)
    if unknown:
        parser.error(f"unrecognized arguments: {' '.join(unknown)}")
    for k, v in vars(args).items():
        if v is None:
            continue
        if k == "no_channels_last":
            config.channels_last = not v
        elif k == "no_aux":
            config.use_aux = not v
        elif k == "no_fused_loss":
            config.fused_loss = not v
        elif k == "no_fused_optimizer":
            config.fused_optimizer = not v
        elif k == "train_mode":  # MyConfig defaults to prediction (reference my_config.py:27)
            config.is_testing = not v
        else:
            setattr(config, k, v)
    return config
