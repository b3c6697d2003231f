"""DistributedStrategy (reference: python/paddle/distributed/fleet/base/distributed_strategy.py,
paddle/fluid/framework/distributed_strategy.proto). Plain attribute bag with the
reference's field names and defaults; (de)serialised to JSON instead of prototxt."""
from __future__ import annotations

import copy
import json

__all__ = ["DistributedStrategy"]

_DEFAULTS = {
    "amp": False,
    "amp_configs": {"init_loss_scaling": 32768.0, "incr_every_n_steps": 1000, "decr_every_n_nan_or_inf": 2,
                    "incr_ratio": 2.0, "decr_ratio": 0.8, "use_dynamic_loss_scaling": True,
                    "custom_white_list": [], "custom_black_list": [], "use_pure_fp16": False, "use_fp16_guard": True,
                    "use_bf16": False},
    "recompute": False,
    "recompute_configs": {"checkpoints": [], "enable_offload": False},
    "sharding": False,
    "sharding_configs": {"sharding_degree": 8, "stage": 1, "segment_broadcast_MB": 32.0, "comm_overlap": True},
    "pipeline": False,
    "pipeline_configs": {"micro_batch_size": 1, "accumulate_steps": 1, "schedule_mode": "1F1B", "p2p_cache_shape": True},
    "tensor_parallel": False,
    "tensor_parallel_configs": {"tensor_parallel_degree": 1, "tensor_init_seed": -1},
    "hybrid_configs": {"dp_degree": -1, "mp_degree": 1, "pp_degree": 1, "sharding_degree": 1},
    "gradient_merge": False,
    "gradient_merge_configs": {"k_steps": 1, "avg": True},
    "lars": False,
    "lars_configs": {"lars_coeff": 0.001, "lars_weight_decay": 0.0005, "epsilon": 0, "exclude_from_weight_decay": []},
    "lamb": False,
    "lamb_configs": {"lamb_weight_decay": 0.01, "exclude_from_weight_decay": []},
    "dgc": False,
    "dgc_configs": {"rampup_begin_step": 0, "rampup_step": 1, "sparsity": [0.999]},
    "localsgd": False,
    "localsgd_configs": {"k_steps": 1, "begin_step": 1},
    "adaptive_localsgd": False,
    "adaptive_localsgd_configs": {"init_k_steps": 1, "begin_step": 1},
    "fp16_allreduce": False,
    "fuse_all_reduce_ops": True,
    "fuse_grad_size_in_MB": 64,
    "last_comm_group_size_MB": 8,
    "find_unused_parameters": False,
    "without_graph_optimization": True,
    "a_sync": False,
    "a_sync_configs": {"k_steps": -1},
    "sync_nccl_allreduce": True,
    "nccl_comm_num": 1,
    "use_hierarchical_allreduce": False,
    "sync_batch_norm": False,
    "auto": False,
    "semi_auto": False,
    "heter_ccl_mode": False,
    "cudnn_exhaustive_search": False,
    "conv_workspace_size_limit": 512,
    "cudnn_batchnorm_spatial_persistent": False,
    "fuse_grad_merge": False,
    "calc_comm_same_stream": False,
    "gradient_scale_configs": {"scale_strategy": "avg"},
    "qat": False,
    "asp": False,
    "elastic": False,
}


class DistributedStrategy:
    def __init__(self):
        object.__setattr__(self, "_d", copy.deepcopy(_DEFAULTS))

    def __getattr__(self, k):
        d = object.__getattribute__(self, "_d")
        if k in d:
            return d[k]
        raise AttributeError(k)

    def __setattr__(self, k, v):
        d = object.__getattribute__(self, "_d")
        if k.endswith("_configs") and k in d and isinstance(v, dict):
            merged = dict(d[k])
            merged.update(v)
            d[k] = merged
        else:
            d[k] = v

    def save_to_prototxt(self, output):
        with open(output, "w") as f:
            json.dump(self._d, f, indent=1, default=str)

    def load_from_prototxt(self, pb_file):
        with open(pb_file) as f:
            self._d.update(json.load(f))

    def __repr__(self):
        return "DistributedStrategy(" + ", ".join(f"{k}={v}" for k, v in self._d.items() if v not in (False, None)) + ")"
