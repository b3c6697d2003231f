"""Loader for the native HIP kernel library (C ABI, ctypes).

The library is built in-tree by ``python -m paddle_hackathon_amd.ops.build``
(or ``__graft_entry__.build()``) into ``paddle_hackathon_amd/_C/libpha_kernels.so``.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_C", "libpha_kernels.so")
if os.environ.get("PHA_KERNELS_LIB"):   # A/B measurements against another in-tree build
    LIB_PATH = os.path.join(os.path.dirname(_HERE), "_C", os.environ["PHA_KERNELS_LIB"])

lib = None
_load_error = None


def _load():
    global lib, _load_error
    if lib is not None:
        return lib
    if not os.path.exists(LIB_PATH):
        _load_error = f"{LIB_PATH} not built (run python -m paddle_hackathon_amd.ops.build)"
        return None
    try:
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - depends on ROCm runtime presence
        _load_error = str(e)
        lib = None
    return lib


def native_available():
    return _load() is not None and torch.cuda.is_available()


def require_native():
    """Called on the first HIP-tensor op: a GPU run without the kernels is an error."""
    if native_available():
        return True
    if os.environ.get("PHA_ALLOW_FALLBACK") == "1":
        return False
    raise RuntimeError(f"paddle_hackathon_amd HIP kernel library unavailable on a GPU run: {_load_error}")


_load()
