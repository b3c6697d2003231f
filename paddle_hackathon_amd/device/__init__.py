"""``paddle.device`` (reference: python/paddle/device/__init__.py). On this framework the
only accelerator is the MI355X (HIP); the ``gpu`` device type maps to it."""
from __future__ import annotations

import torch

from ..framework.core import (set_device, get_device, XPUPlace, IPUPlace, MLUPlace, CPUPlace, CUDAPlace,  # noqa: F401
                              _gpu_available)
from . import cuda  # noqa: F401

__all__ = ["get_cudnn_version", "set_device", "get_device", "XPUPlace", "IPUPlace", "MLUPlace",
           "is_compiled_with_xpu", "is_compiled_with_ipu", "is_compiled_with_cinn", "is_compiled_with_cuda",
           "is_compiled_with_rocm", "is_compiled_with_npu", "is_compiled_with_mlu", "get_all_device_type",
           "get_all_custom_device_type", "get_available_device", "get_available_custom_device"]


def get_cudnn_version():
    """MIOpen version as an int (major*1000+minor*100+patch), or None without a GPU."""
    if not _gpu_available():
        return None
    v = torch.backends.cudnn.version() if torch.backends.cudnn.is_available() else None
    return v


def is_compiled_with_cuda():
    return _gpu_available()


def is_compiled_with_rocm():
    return torch.version.hip is not None


def is_compiled_with_xpu():
    return False


is_compiled_with_ipu = is_compiled_with_npu = is_compiled_with_mlu = is_compiled_with_cinn = is_compiled_with_xpu


def get_all_device_type():
    return ["cpu"] + (["gpu"] if _gpu_available() else [])


def get_all_custom_device_type():
    return []


def get_available_device():
    out = ["cpu"]
    if _gpu_available():
        out += [f"gpu:{i}" for i in range(torch.cuda.device_count())]
    return out


def get_available_custom_device():
    return []
