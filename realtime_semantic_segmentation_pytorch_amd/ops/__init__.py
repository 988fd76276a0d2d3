"""Hand-written HIP/CDNA4 operators and their autograd wrappers.

Every public op dispatches to the in-tree HIP extension for GPU tensors and to
an equivalent PyTorch formulation for CPU tensors (see ``_ext.py``).
"""
from ._ext import load, use_hip, hip_disabled, library_path
from .interp import (interpolate, final_upsample, defer_final_upsample, DeferredLogits,
                     materialize)
from .seg_loss import (seg_cross_entropy, seg_cross_entropy_reference, MODE_OHEM, MODE_MEAN,
                       MODE_SUM)
from .kd import kd_kl_div, kd_kl_div_reference
from .bn import (bn_act, bn_stats_begin, bias_add, act_code as bn_act_code, fused_ok as bn_fused_ok, convert_batchnorm,
                 FusedBatchNorm2d, FusedSyncBatchNorm)
from .detail import detail_loss, detail_loss_reference, detail_target_reference
from .postprocess import colorize, colorize_reference
from .confmat import confusion_matrix, confusion_matrix_reference
from .concat import ConcatSink, cat_bn_act
from .dwconv import DepthwiseConv2d, convert_depthwise, depthwise_ok, dw_conv2d, dw_conv_bn_eval, dw_conv_bn_stats
from .pool import (avg_pool2d, max_pool2d, adaptive_avg_pool2d, convert_pooling, AvgPool2d, MaxPool2d,
                   AdaptiveAvgPool2d, MaxUnpool2d, max_pool2d_with_indices, max_unpool2d, AdaptiveMaxPool2d,
                   adaptive_max_pool2d)
from .tapconv import TapConv2d, convert_tap_convs, tap_conv2d, tapconv_ok
from .dilated import (DilatedGroupConv2d, convert_dilated_group_convs, dilated_group_conv2d, dilated_group_ok,
                      PrunedConv2d, convert_pruned_convs, pruned_conv2d, has_dead_taps)
from .optim import FusedAdam, FusedAdamW, FusedSGD
from .conv import (conv_ok, conv_bn_stats, stem_store_skippable, twin_conv_bn_stats, conv_bn_act_eval, conv_bn_act, conv_forward, RoutedConv2d, GroupedConv2d,
                   convert_routed_convs, invalidate_weight_shadows)
from .deconv import TransposedConv2d, conv_transpose2d, convert_transposed_convs, deconv_ok
from .gate import gate, gate_reference
from .act import activation, convert_activations
from .shuffle import channel_shuffle, convert_pixel_shuffle, pixel_shuffle, pixel_unshuffle
from .augment import AugmentSpec, augment_batch, augment_reference, draw_params
from .streams import concurrent_branches

__all__ = [
    "load", "use_hip", "hip_disabled", "library_path",
    "interpolate", "final_upsample", "defer_final_upsample", "DeferredLogits", "materialize",
    "seg_cross_entropy", "seg_cross_entropy_reference", "MODE_OHEM", "MODE_MEAN", "MODE_SUM",
    "colorize", "colorize_reference", "kd_kl_div", "kd_kl_div_reference", "detail_loss", "detail_loss_reference", "detail_target_reference", "confusion_matrix", "confusion_matrix_reference",
    "DepthwiseConv2d", "convert_depthwise", "depthwise_ok", "dw_conv2d", "dw_conv_bn_eval", "dw_conv_bn_stats",
    "avg_pool2d", "max_pool2d", "adaptive_avg_pool2d", "convert_pooling", "AvgPool2d", "MaxPool2d",
    "AdaptiveAvgPool2d", "AdaptiveMaxPool2d", "adaptive_max_pool2d", "MaxUnpool2d", "max_pool2d_with_indices", "max_unpool2d", "TapConv2d", "convert_tap_convs", "tap_conv2d", "tapconv_ok",
    "DilatedGroupConv2d", "convert_dilated_group_convs", "dilated_group_conv2d", "dilated_group_ok",
    "PrunedConv2d", "convert_pruned_convs", "pruned_conv2d", "has_dead_taps",
    "FusedSGD", "FusedAdam", "FusedAdamW", "conv_ok", "conv_bn_stats", "stem_store_skippable", "twin_conv_bn_stats", "conv_bn_act_eval", "conv_bn_act", "conv_forward", "RoutedConv2d", "GroupedConv2d", "convert_routed_convs", "invalidate_weight_shadows",
    "TransposedConv2d", "conv_transpose2d", "convert_transposed_convs", "deconv_ok", "gate", "gate_reference", "activation", "convert_activations", "channel_shuffle", "convert_pixel_shuffle", "pixel_shuffle", "pixel_unshuffle", "AugmentSpec", "augment_batch", "augment_reference", "draw_params",
    "concurrent_branches", "ConcatSink", "cat_bn_act", "bn_act", "bn_stats_begin", "bias_add", "bn_act_code", "bn_fused_ok", "convert_batchnorm", "FusedBatchNorm2d", "FusedSyncBatchNorm",
]
