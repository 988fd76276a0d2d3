"""User override config (parity: reference configs/my_config.py:4-50)."""
from .base_config import BaseConfig


class MyConfig(BaseConfig):
    def __init__(self):
        super().__init__()
        # dataset
        self.dataset = "cityscapes"
        self.data_root = "/path/to/your/dataset"
        self.num_class = 19

        # model
        self.model = "bisenetv2"

        # training
        self.total_epoch = 200
        self.train_bs = 8
        self.loss_type = "ohem"
        self.optimizer_type = "adam"
        self.logger_name = "seg_trainer"
        self.use_aux = True

        # validating
        self.val_bs = 10

        # testing
        self.is_testing = True
        self.test_bs = 8
        self.test_data_folder = "/path/to/your/test/folder"
        self.load_ckpt_path = "/path/to/your/inference/checkpoint"
        self.save_mask = True

        # training setting
        self.use_ema = False

        # augmentation
        self.crop_size = 768
        self.randscale = [-0.5, 1.0]
        self.scale = 1.0
        self.brightness = 0.5
        self.contrast = 0.5
        self.saturation = 0.5
        self.h_flip = 0.5

        # knowledge distillation
        self.kd_training = False
        self.teacher_ckpt = "/path/to/your/teacher/checkpoint"
        self.teacher_model = "smp"
        self.teacher_encoder = "resnet101"
        self.teacher_decoder = "deeplabv3p"
