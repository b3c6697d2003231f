"""Global flags (reference: paddle/fluid/platform/flags.cc, python/paddle/fluid/framework.py:set_flags)."""
from __future__ import annotations

import os

__all__ = ["set_flags", "get_flags", "flag"]

_FLAGS = {
    "FLAGS_check_nan_inf": False,
    "FLAGS_check_nan_inf_level": 0,
    "FLAGS_cudnn_deterministic": False,
    "FLAGS_use_autotune": False,
    "FLAGS_eager_delete_tensor_gb": 0.0,
    "FLAGS_fraction_of_gpu_memory_to_use": 0.92,
    "FLAGS_allocator_strategy": "auto_growth",
    "FLAGS_embedding_deterministic": False,
    "FLAGS_cudnn_exhaustive_search": False,
    "FLAGS_conv_workspace_size_limit": 512,
    "FLAGS_benchmark": False,
    "FLAGS_use_hip_graph": False,
}
for _k in list(_FLAGS):
    if _k in os.environ:
        v = os.environ[_k]
        d = _FLAGS[_k]
        _FLAGS[_k] = (v.lower() in ("1", "true")) if isinstance(d, bool) else type(d)(v)


def _sync_mode():
    from .core import _mode
    _mode.check_nan_inf = bool(_FLAGS["FLAGS_check_nan_inf"])


def set_flags(flags):
    for k, v in flags.items():
        _FLAGS[k] = v
        if k == "FLAGS_check_nan_inf":
            _sync_mode()
        if k == "FLAGS_cudnn_deterministic":
            import torch
            torch.backends.cudnn.deterministic = bool(v)


def get_flags(flags):
    if isinstance(flags, str):
        flags = [flags]
    return {k: _FLAGS.get(k) for k in flags}


def flag(name, default=None):
    return _FLAGS.get(name, default)


if _FLAGS["FLAGS_check_nan_inf"]:
    _sync_mode()
