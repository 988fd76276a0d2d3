"""Attribute-bag configuration (parity: reference configs/base_config.py:1-109).

Every knob of the reference exists here with the same name and default.  Fields
the reference reads but never defines (``reduction``,
``step_size``, ``train_size``, ``test_size``, ``logger_name``; ``data_root`` vs
``dataroot``) get defaults, and the MI355X-specific knobs are grouped at the
end (all default to the behaviour a reference user expects).
"""
from __future__ import annotations


class BaseConfig:
    def __init__(self):
        # ---- dataset
        self.dataset = None
        self.dataroot = None
        self.data_root = None            # alias actually read by the datasets
        self.num_class = -1
        self.ignore_index = 255

        # ---- model
        self.model = None
        self.encoder = None
        self.decoder = None
        self.encoder_weights = "imagenet"
        # choose among a model family's variants (None = the reference default;
        # e.g. ddrnet: 'DDRNet-23-slim' | 'DDRNet-23' | 'DDRNet-39')
        self.arch_type = None
        self.encoder_type = None         # stdc / ppliteseg: 'stdc1' | 'stdc2'
        self.backbone_type = None        # resnet-based models: 'resnet18' ...

        # ---- detail head (STDC)
        self.use_detail_head = False
        self.detail_thrs = 0.1
        self.detail_loss_coef = 1.0
        self.dice_loss_coef = 1.0
        self.bce_loss_coef = 1.0

        # ---- training
        self.total_epoch = 200
        self.base_lr = 0.01
        self.train_bs = 16               # per GPU
        self.use_aux = False
        self.aux_coef = None
        self.logger_name = "seg_trainer"

        # ---- validating
        self.val_bs = 16                 # per GPU
        self.begin_val_epoch = 0
        self.val_interval = 1

        # ---- testing
        self.is_testing = False
        self.test_bs = 16
        self.test_data_folder = None
        self.colormap = "cityscapes"
        self.save_mask = True
        self.blend_prediction = True
        self.blend_alpha = 0.3

        # ---- loss
        self.loss_type = "ohem"
        self.class_weights = None
        self.ohem_thrs = 0.7
        self.reduction = "mean"

        # ---- scheduler
        self.lr_policy = "cos_warmup"
        self.warmup_epochs = 3
        self.step_size = 30              # epochs, for lr_policy='step'

        # ---- optimizer
        self.optimizer_type = "sgd"
        self.momentum = 0.9
        self.weight_decay = 1e-4

        # ---- monitoring
        self.save_ckpt = True
        self.save_dir = "save"
        self.use_tb = True
        self.tb_log_dir = None
        self.ckpt_name = None

        # ---- training setting
        self.amp_training = False
        self.resume_training = True
        self.load_ckpt = True
        self.load_ckpt_path = None
        self.base_workers = 8
        self.random_seed = 1
        self.use_ema = False

        # ---- augmentation
        self.crop_size = 512
        self.crop_h = None
        self.crop_w = None
        self.scale = 1.0
        self.randscale = 0.0
        self.brightness = 0.0
        self.contrast = 0.0
        self.saturation = 0.0
        self.h_flip = 0.0
        self.v_flip = 0.0
        self.train_size = None           # custom dataset ResizeToSquare size
        self.test_size = None

        # ---- DDP
        self.synBN = True

        # ---- knowledge distillation
        self.kd_training = False
        self.teacher_ckpt = ""
        self.teacher_model = "smp"
        self.teacher_encoder = None
        self.teacher_decoder = None
        self.kd_loss_type = "kl_div"
        self.kd_loss_coefficient = 1.0
        self.kd_temperature = 4.0

        # ---- MI355X execution knobs (not in the reference)
        self.amp_dtype = "bf16"          # autocast dtype when amp_training: 'bf16' | 'fp16'
        self.channels_last = True        # NHWC activations (MIOpen/HIP kernels prefer it)
        self.cudnn_benchmark = False     # MIOpen find mode (exhaustive solver search) for convs left on MIOpen; opt-in (utils/runtime.py)
        self.deterministic = False       # bit-reproducible steps across processes: no conv timing, MIOpen deterministic solvers (utils/runtime.py)
        self.fused_loss = True           # fold the final upsample into the HIP loss kernel
        self.fused_optimizer = True      # HIP multi-tensor optimizer step that also writes the EMA
        self.hip_depthwise = True        # depth-wise convs on the HIP kernels (else MIOpen)
        self.hip_pooling = True          # avg / max / adaptive pooling on the HIP kernels
        self.hip_activations = True      # PReLU / ELU / SELU / Hardswish / SiLU / ... on the HIP kernels
        self.ddp_bucket_mb = 32          # RCCL all-reduce bucket: ~3 buckets for DDRNet-23 (84 MB), overlapped with backward
        self.ddp_static_graph = True
        self.pg_timeout_s = 600          # collective timeout: a hung rank fails the job (non-zero exit) instead of holding the node
        self.syncbn_group = "own"        # SyncBN statistics on their own communicator ('own') or DDP's ('default')
        self.spawn_procs = None          # main.py without torchrun: worker processes (None: one per visible GPU)
        self.graph_step = False          # replay forward+loss+backward from one captured HIP graph (small batches)
        self.graph_warmup = 3            # eager steps per input shape before the capture
        self.kd_teacher_graph = True     # KD teacher as a captured HIP graph with pre-cast weights
        self.gpu_aug = False             # training augmentation on the GPU (ops/augment.py): workers only decode
        self.synthetic_data = False      # device-generated synthetic batches (benchmarks)
        self.synthetic_len = 64          # images per epoch of the synthetic dataset
        self.synthetic_size = None       # (H, W) of synthetic images (default: crop)
        self.synthetic_learnable = False  # labels a function of the image (colour-coded blocks)
        self.synthetic_cell = 32         # block size (pixels) of the learnable synthetic task
        self.max_train_itrs = None       # stop an epoch early (smoke runs)
        self.log_interval = 20           # iterations between host-synced loss logs
        self.device = None               # force 'cpu' / 'cuda'

    def init_dependent_config(self):
        if self.data_root is None and self.dataroot is not None:
            self.data_root = self.dataroot
        if self.dataroot is None and self.data_root is not None:
            self.dataroot = self.data_root
        if self.load_ckpt_path is None and not self.is_testing:
            self.load_ckpt_path = f"{self.save_dir}/last.pth"
        if self.tb_log_dir is None:
            self.tb_log_dir = f"{self.save_dir}/tb_logs/"
        if self.crop_h is None:
            self.crop_h = self.crop_size
        if self.crop_w is None:
            self.crop_w = self.crop_size
        return self
