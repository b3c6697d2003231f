"""``paddle.utils`` (reference: python/paddle/utils/{deprecated,lazy_import,install_check,
dlpack,unique_name,download}.py, utils/cpp_extension)."""
from __future__ import annotations

import functools
import importlib
import warnings

from . import unique_name  # noqa: F401
from . import dlpack  # noqa: F401
from . import download  # noqa: F401

__all__ = ["deprecated", "run_check", "require_version", "try_import"]


def deprecated(update_to="", since="", reason="", level=0):
    """Decorator emitting a DeprecationWarning (level 2 raises) on call."""
    def deco(fn):
        msg = f"API \"{fn.__module__}.{fn.__name__}\" is deprecated"
        if since:
            msg += f" since {since}"
        if update_to:
            msg += f", and will be removed in future versions. Please use \"{update_to}\" instead"
        if reason:
            msg += f". Reason: {reason}"

        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            if level == 2:
                raise RuntimeError(msg)
            if level == 1:
                warnings.warn(msg, category=DeprecationWarning, stacklevel=2)
            return fn(*args, **kwargs)
        wrapper.__doc__ = (fn.__doc__ or "") + f"\n\nWarning: {msg}"
        return wrapper
    return deco


def _parse(v):
    out = []
    for p in str(v).split("."):
        digits = "".join(c for c in p if c.isdigit())
        out.append(int(digits) if digits else 0)
    return (out + [0, 0, 0, 0])[:4]


def require_version(min_version, max_version=None):
    """Raise if the installed framework version is outside [min_version, max_version]."""
    from .. import __version__
    if not isinstance(min_version, str):
        raise TypeError(f"min_version must be str, got {type(min_version)}")
    cur = _parse(__version__)
    if __version__.startswith("0.0.0"):
        return
    if cur < _parse(min_version) or (max_version is not None and cur > _parse(max_version)):
        raise Exception(f"VersionError: installed version {__version__} not in [{min_version}, {max_version}]")


def try_import(module_name):
    try:
        return importlib.import_module(module_name)
    except ImportError as e:
        raise ImportError(f"Failed importing {module_name}. This likely means that some modules require "
                          f"additional dependencies that have to be manually installed.") from e


def run_check():
    """Install check: one tiny train step on the MI355X (or CPU), and on all visible GPUs via DataParallel
    if more than one is present (reference: utils/install_check.py:223)."""
    import numpy as np
    import torch
    from .. import nn, optimizer, to_tensor
    dev = "gpu" if torch.cuda.is_available() else "cpu"
    print(f"Running verify PaddlePaddle-AMD program on {dev} ... ")
    lin = nn.Linear(2, 4)
    opt = optimizer.SGD(learning_rate=1e-3, parameters=lin.parameters())
    x = to_tensor(np.random.rand(8, 2).astype("float32"))
    loss = lin(x).mean()
    loss.backward()
    opt.step()
    if dev == "gpu":
        from ..ops import native_available
        if not native_available():
            raise RuntimeError("MI355X visible but the gfx950 kernel library failed to load")
    print("PaddlePaddle-AMD works well on 1 " + dev + ".")
    print("PaddlePaddle-AMD is installed successfully! Let's start deep learning with PaddlePaddle-AMD now.")
