"""paddle_hackathon_amd — an MI355X-native deep-learning framework with PaddlePaddle's
``paddle.*`` API (reference: ccw1996/Paddle_hackathon, python/paddle/__init__.py).

Compute path: PyTorch-ROCm tensors/autograd + hand-written gfx950 HIP kernels
(``paddle_hackathon_amd.ops``) + RCCL over xGMI (``paddle_hackathon_amd.distributed``).
Use it as ``import paddle_hackathon_amd as paddle``.
"""
from __future__ import annotations

import importlib
import sys as _sys

__version__ = "0.1.0"
version = type("version", (), {"full_version": __version__, "major": "0", "minor": "1", "patch": "0",
                                "rc": "0", "istaged": True, "commit": "mi355x", "with_mkl": "OFF",
                                "show": staticmethod(lambda: print(__version__)), "cuda": staticmethod(lambda: "False"),
                                "cudnn": staticmethod(lambda: "False")})

from .framework import core as _core  # noqa: E402
from .framework.core import (  # noqa: E402,F401
    Tensor, Parameter, ParamBase, EagerParamBase, VarBase, to_tensor, is_tensor, CPUPlace, CUDAPlace,
    CUDAPinnedPlace, XPUPlace, NPUPlace, MLUPlace, IPUPlace, CustomPlace, set_device, get_device,
    set_default_dtype, get_default_dtype, in_dynamic_mode, dtype,
    bool_ as bool, uint8, int8, int16, int32, int64, float16, bfloat16, float32, float64, complex64, complex128,
)
from .framework.param_attr import ParamAttr, WeightNormParamAttr  # noqa: E402,F401
from .framework.io import save, load  # noqa: E402,F401
from .framework.flags import set_flags, get_flags  # noqa: E402,F401
from .tensor import *  # noqa: E402,F401,F403
from .tensor import getitem as _getitem  # noqa: E402,F401
from .tensor.random import seed, get_cuda_rng_state, set_cuda_rng_state, get_rng_state, set_rng_state  # noqa: E402,F401
from .tensor.creation import create_parameter  # noqa: E402,F401
from .autograd import grad, no_grad, enable_grad, set_grad_enabled, is_grad_enabled  # noqa: E402,F401
from . import ops  # noqa: E402,F401
from . import nn  # noqa: E402,F401
from . import optimizer  # noqa: E402,F401
from . import regularizer  # noqa: E402,F401
from . import amp  # noqa: E402,F401
from . import io  # noqa: E402,F401
from . import autograd  # noqa: E402,F401
from . import parallel  # noqa: E402,F401
from .parallel import DataParallel  # noqa: E402,F401

distributed = parallel
_sys.modules[__name__ + ".distributed"] = parallel
for _k, _v in list(_sys.modules.items()):
    if _k.startswith(__name__ + ".parallel."):
        _sys.modules[__name__ + ".distributed." + _k[len(__name__ + ".parallel."):]] = _v

# lazily imported sub-packages (keeps `import paddle_hackathon_amd` light)
_LAZY = {
    "static": ".static", "jit": ".jit", "vision": ".vision", "text": ".text", "metric": ".metric",
    "hapi": ".hapi", "callbacks": ".hapi.callbacks", "profiler": ".profiler", "distribution": ".distribution",
    "sparse": ".sparse", "incubate": ".incubate", "device": ".device", "utils": ".utils", "linalg": ".linalg",
    "fft": ".fft", "signal": ".signal", "inference": ".inference", "onnx": ".onnx", "hub": ".hub",
    "models": ".models", "sysconfig": ".sysconfig", "dataset": ".dataset", "reader": ".reader", "fluid": ".fluid",
    "batch": ".reader", "Model": ".hapi", "summary": ".hapi", "flops": ".hapi", "compat": ".compat",
    "enable_static": ".static", "disable_static": ".static", "cost_model": ".cost_model",
}


def __getattr__(name):
    if name in _LAZY:
        try:
            mod = importlib.import_module(_LAZY[name], __name__)
        except ImportError as e:
            raise AttributeError(f"paddle_hackathon_amd.{name} unavailable: {e}") from e
        if name in ("Model", "summary", "flops", "enable_static", "disable_static", "batch"):
            return getattr(mod, name)
        globals()[name] = mod
        return mod
    raise AttributeError(f"module 'paddle_hackathon_amd' has no attribute {name!r}")


def is_compiled_with_cuda():
    """True when an MI355X (HIP device) is usable — Paddle code gates GPU paths on this."""
    return _core._gpu_available()


def is_compiled_with_rocm():
    return True


def is_compiled_with_xpu():
    return False


def is_compiled_with_npu():
    return False


def is_compiled_with_mlu():
    return False


def is_compiled_with_ipu():
    return False


def is_compiled_with_cinn():
    return False


def disable_signal_handler():
    pass


def get_cudnn_version():
    return None


def monkey_patch_variable():
    pass


from .framework.core import set_printoptions  # noqa: E402,F401


def check_shape(shape):
    """Validate a shape argument: list/tuple of ints (>= -1) or Tensors, or an int Tensor
    (reference: fluid/layers/utils.py:check_shape)."""
    if isinstance(shape, Tensor):
        if shape.dtype not in (int32, int64):
            raise TypeError("shape Tensor must be int32 or int64")
        return
    if not isinstance(shape, (list, tuple)):
        raise TypeError(f"shape must be list/tuple/Tensor, got {type(shape)}")
    for e in shape:
        if isinstance(e, Tensor):
            continue
        if not isinstance(e, int):
            raise TypeError(f"All elements in ``shape`` must be integers, got {type(e)}")
        if e < -1:
            raise ValueError("All elements in ``shape`` must be positive when it's a list or tuple")


def monkey_patch_math_varbase():
    pass
