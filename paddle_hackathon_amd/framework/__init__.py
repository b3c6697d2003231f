"""``paddle.framework`` (reference: python/paddle/framework/__init__.py): ParamAttr, the default
dtype, seeds and the core module."""
from .core import get_default_dtype, set_default_dtype  # noqa: F401
from .param_attr import ParamAttr  # noqa: F401


def __getattr__(name):   # seed / random / rng states: from tensor.random (imported after this package)
    if name in ("seed", "get_cuda_rng_state", "set_cuda_rng_state"):
        from ..tensor import random as _r
        return getattr(_r, name)
    if name == "random":
        import importlib
        return importlib.import_module(".random", __name__)
    raise AttributeError(name)
