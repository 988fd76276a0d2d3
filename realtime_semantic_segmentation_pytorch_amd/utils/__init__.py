from .utils import (mkdir, set_seed, get_writer, get_logger, save_config, log_config, get_colormap,
                    JsonlWriter)
from .metrics import SegMetrics, get_seg_metrics
from .optim import get_optimizer, get_scheduler, ModelEmaV2, get_ema_model
from ..parallel import (is_parallel, de_parallel, set_device, parallel_model, destroy_ddp_process,
                        sampler_set_epoch)
