from .ddp import (is_parallel, de_parallel, dist_env, is_dist, get_rank, get_world_size, barrier,
                  set_device, parallel_model, destroy_ddp_process, sampler_set_epoch,
                  all_reduce_mean)

__all__ = ["is_parallel", "de_parallel", "dist_env", "is_dist", "get_rank", "get_world_size",
           "barrier", "set_device", "parallel_model", "destroy_ddp_process", "sampler_set_epoch",
           "all_reduce_mean"]
