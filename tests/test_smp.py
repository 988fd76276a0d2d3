"""SMP-compatible encoder/decoder models (config.model='smp') and the KD teacher (CPU).

segmentation_models_pytorch is not installed, so parity with real SMP is
"parity unpinned"; these tests pin the module layout we rely on (SMP key
prefixes, parameter counts of well-known SMP configurations, output shapes,
encoder strides / dilation rule) and the teacher-loading path.
"""
import os

import pytest
import torch

from realtime_semantic_segmentation_pytorch_amd import ops
from realtime_semantic_segmentation_pytorch_amd.configs import BaseConfig
from realtime_semantic_segmentation_pytorch_amd.models import get_model, get_teacher_model
from realtime_semantic_segmentation_pytorch_amd.models.smp import DECODER_HUB, build_smp_model, get_encoder

# parameter counts (M) of SMP models with ResNet-18 encoders and 19 classes
PARAMS_R18 = {"deeplabv3": 15.904, "deeplabv3p": 12.334, "fpn": 13.050, "linknet": 11.664, "manet": 21.678,
              "pan": 11.373, "pspnet": 11.413, "unet": 14.331, "unetpp": 15.973}


@pytest.mark.parametrize("decoder", sorted(DECODER_HUB))
def test_smp_decoder_shapes_keys_params(decoder):
    m = build_smp_model(decoder, "resnet18", None, 19)
    n = sum(p.numel() for p in m.parameters()) / 1e6
    assert abs(n - PARAMS_R18[decoder]) < 1e-3
    keys = list(m.state_dict())
    assert keys[0] == "encoder.conv1.weight" and keys[-1] == "segmentation_head.0.bias"
    assert all(k.split(".")[0] in ("encoder", "decoder", "segmentation_head") for k in keys)
    x = torch.randn(2, 3, 128, 128)  # PAN's pyramid needs >= 128 px
    m.train()
    y = m(x)
    assert y.shape == (2, 19, 128, 128)
    y.float().mean().backward()
    m.eval()
    with torch.no_grad():
        assert m(x).shape == (2, 19, 128, 128)


def test_smp_deferred_head_matches_full_output():
    m = build_smp_model("deeplabv3p", "resnet18", None, 19).eval()
    x = torch.randn(1, 3, 64, 128)
    ref = m(x)
    with ops.defer_final_upsample():
        d = m(x)
    assert isinstance(d, ops.DeferredLogits) and tuple(d.logits.shape[2:]) == (16, 32)
    torch.testing.assert_close(d.materialize(), ref, atol=1e-5, rtol=1e-5)


def test_encoder_strides_and_smp_dilation_rule():
    e = get_encoder("resnet50", depth=5, output_stride=8)
    feats = e(torch.randn(1, 3, 64, 64))
    assert [f.shape[1] for f in feats] == [3, 64, 256, 512, 1024, 2048]
    assert [f.shape[2] for f in feats] == [64, 32, 16, 8, 8, 8]
    # SMP rule: EVERY conv of a dilated stage gets the stage's rate (not torchvision's first-block rule)
    assert e.layer3[0].conv2.dilation == (2, 2) and e.layer4[0].conv2.dilation == (4, 4)
    assert e.layer4[0].downsample[0].stride == (1, 1)
    m = get_encoder("mobilenet_v2", depth=5)
    assert [f.shape[1] for f in m(torch.randn(1, 3, 64, 64))] == [3, 16, 24, 32, 96, 1280]


def test_unsupported_encoders_raise():
    with pytest.raises(ValueError):  # SMP: MiT has no dilated mode and only 3 input channels
        get_encoder("mit_b0", output_stride=16)
    with pytest.raises(ValueError):
        get_encoder("mit_b0", in_channels=4)
    with pytest.raises(ValueError):
        build_smp_model("unetpp", "mit_b0", None, 19)
    with pytest.raises(ValueError):
        build_smp_model("nope", "resnet18", None, 19)


def test_get_model_smp_and_teacher_roundtrip(tmp_path):
    c = BaseConfig()
    c.model, c.encoder, c.decoder, c.encoder_weights, c.num_class = "smp", "resnet18", "unet", None, 19
    c.use_aux = c.use_detail_head = False
    assert get_model(c).__class__.__name__ == "Unet"
    # teacher: {'state_dict': smp_state} checkpoint, loaded with weights_only=True
    t = build_smp_model("deeplabv3p", "resnet18", None, 19)
    path = os.path.join(tmp_path, "teacher.pth")
    torch.save({"state_dict": t.state_dict()}, path)
    c.kd_training, c.teacher_ckpt, c.teacher_encoder, c.teacher_decoder = True, path, "resnet18", "deeplabv3p"
    teacher = get_teacher_model(c, torch.device("cpu"))
    assert not teacher.training
    assert all(not p.requires_grad for p in teacher.parameters())
    for k, v in t.state_dict().items():
        assert torch.equal(teacher.state_dict()[k], v)


@pytest.mark.gpu
@pytest.mark.parametrize("decoder", sorted(DECODER_HUB))
def test_smp_bf16_train_step_gpu(decoder):
    from realtime_semantic_segmentation_pytorch_amd.core.loss import SegCELoss

    m = build_smp_model(decoder, "resnet18", None, 19).cuda().to(memory_format=torch.channels_last).train()
    x = torch.randn(2, 3, 128, 256, device="cuda").contiguous(memory_format=torch.channels_last)
    labels = torch.randint(0, 19, (2, 128, 256), device="cuda", dtype=torch.uint8)
    with torch.autocast("cuda", dtype=torch.bfloat16), ops.defer_final_upsample():
        loss = SegCELoss(ops.MODE_OHEM, 0.7)(m(x), labels)
    loss.backward()
    assert torch.isfinite(loss)
    assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)


def test_mit_encoder_contract():
    """SMP's MixVisionTransformerEncoder contract: [x, 0-channel stride-2 placeholder, /4, /8, /16,
    /32] with MiT-B0's widths; SMP checkpoint key layout (incl. the unused ImageNet head)."""
    e = get_encoder("mit_b0", depth=5)
    feats = e(torch.randn(2, 3, 64, 96))
    assert [tuple(f.shape[1:]) for f in feats] == [(3, 64, 96), (0, 32, 48), (32, 16, 24), (64, 8, 12),
                                                   (160, 4, 6), (256, 2, 3)]
    assert e.out_channels == (3, 0, 32, 64, 160, 256)
    keys = set(e.state_dict())
    for k in ("patch_embed1.proj.weight", "patch_embed4.norm.bias", "block1.1.attn.sr.weight",
              "block1.0.attn.norm.weight", "block3.1.mlp.dwconv.dwconv.weight", "block4.1.attn.kv.weight",
              "norm4.weight", "head.weight"):
        assert k in keys, k
    assert not any(k.startswith("block4.0.attn.sr") for k in keys)  # stage 4: sr ratio 1
    assert len(e.block3) == 2 and len(get_encoder("mit_b2").block3) == 6
    # an ImageNet checkpoint without its classifier still loads strictly
    sd = {k: v for k, v in e.state_dict().items() if not k.startswith("head.")}
    e.load_state_dict(sd)


@pytest.mark.parametrize("decoder", ["unet", "fpn", "pspnet", "manet", "pan"])
def test_mit_with_supported_decoders(decoder):
    torch.manual_seed(0)
    m = build_smp_model(decoder, "mit_b0", None, 19).train()
    hw = 256 if decoder == "pan" else 64  # PAN's FPA pools the stride-32 map 8x further
    x = torch.randn(2, 3, hw, hw)
    y = m(x)
    assert y.shape == (2, 19, hw, hw)
    y.float().square().mean().backward()
    assert m.encoder.patch_embed1.proj.weight.grad is not None
    if decoder == "pan":  # reference models/__init__.py:69-73: MiT + PAN at encoder output stride 32
        assert m.encoder.output_stride == 32


def test_resnext_encoder_matches_torchvision_layout():
    e = get_encoder("resnext50_32x4d", depth=5)
    assert e.layer1[0].conv2.groups == 32 and e.layer1[0].conv2.in_channels == 128
    assert e.layer4[0].conv2.out_channels == 1024 and e.layer4[0].conv3.out_channels == 2048
    # torchvision resnext50_32x4d has 25,028,904 parameters, 2,049,000 of them in the fc head
    assert sum(p.numel() for p in e.parameters()) == 25_028_904 - 2_049_000
    feats = e(torch.randn(1, 3, 64, 64))
    assert [f.shape[1] for f in feats] == [3, 64, 256, 512, 1024, 2048]
    assert get_encoder("resnext101_32x8d").layer3[22].conv2.groups == 32


# encoders beyond ResNet / MobileNetV2 / MiT (models/smp/encoders_extra.py): parameter counts of
# the published backbones without their classifier heads (torchvision vgg / densenet,
# EfficientNet-PyTorch, pretrainedmodels SENet) and SMP's stage channels
_EXTRA = {"vgg16": 14.71, "vgg19_bn": 20.04, "densenet121": 6.95, "densenet161": 26.47, "densenet201": 18.09,
          "efficientnet-b0": 4.01, "efficientnet-b4": 17.55, "efficientnet-b7": 63.79, "se_resnet50": 26.04,
          "se_resnext50_32x4d": 25.51}


@pytest.mark.parametrize("name", sorted(_EXTRA))
def test_extra_encoders_params_and_stages(name):
    from realtime_semantic_segmentation_pytorch_amd.models.smp import get_encoder

    enc = get_encoder(name)
    assert abs(sum(p.numel() for p in enc.parameters()) / 1e6 - _EXTRA[name]) < 0.01
    x = torch.randn(1, 3, 64, 64)
    with torch.no_grad():
        feats = enc(x)
    assert [f.shape[1] for f in feats] == list(enc.out_channels)
    assert [f.shape[-1] for f in feats] == [64 >> i for i in range(6)]


@pytest.mark.parametrize("enc", ["efficientnet-b0", "densenet121", "se_resnext50_32x4d", "vgg11_bn"])
def test_unet_with_extra_encoder_trains(enc):
    from realtime_semantic_segmentation_pytorch_amd.models.smp import build_smp_model

    m = build_smp_model("unet", enc, None, 19).train()
    y = m(torch.randn(2, 3, 64, 64))
    assert y.shape == (2, 19, 64, 64)
    y.float().mean().backward()
    if enc.startswith("vgg"):  # SMP's center block for VGG encoders: deepest width, two Conv2dReLU
        sd = m.state_dict()
        c = m.encoder.out_channels[-1]
        assert sd["decoder.center.0.0.weight"].shape == (c, c, 3, 3)
        assert sd["decoder.center.1.0.weight"].shape == (c, c, 3, 3)
        assert "decoder.center.1.1.running_var" in sd
    # EfficientNet keeps its (unused) _conv_head / _bn1 in the state dict, as SMP does
    missing = [n for n, p in m.named_parameters() if p.grad is None and "_conv_head" not in n and ".encoder._bn1" not in
               "." + n]
    assert not missing, missing[:5]


def test_unetplusplus_vgg_center_keys_unused():
    """SMP's U-Net++ builds the VGG center block (its state-dict keys) but its forward skips it."""
    from realtime_semantic_segmentation_pytorch_amd.models.smp import build_smp_model

    m = build_smp_model("unetpp", "vgg11_bn", None, 19).train()
    assert "decoder.center.0.0.weight" in m.state_dict()
    m(torch.randn(2, 3, 64, 64)).float().mean().backward()
    assert all(p.grad is None for n, p in m.named_parameters() if n.startswith("decoder.center."))
    assert all(p.grad is not None for n, p in m.named_parameters() if n.startswith("decoder.blocks."))
