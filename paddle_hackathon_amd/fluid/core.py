"""``paddle.fluid.core`` (reference: python/paddle/fluid/core.py, the pybind ``core`` module:
paddle/fluid/pybind/tensor_py.h LoDTensor, pybind.cc Scope / places / VarDesc).

There is no separate C++ tensor type here: ``LoDTensor`` is the framework ``Tensor`` plus a
level-of-detail offset table (``_lod``). ``set(array, place)`` loads data, ``lod()`` /
``set_lod()`` / ``recursive_sequence_lengths()`` manage the offsets, and the fluid sequence
layers (fluid/layers/sequence_lod.py) read them to cut the flat [sum(len), ...] rows into
sequences. A plain ``Tensor`` given ``_lod`` the same way is equally a LoD tensor.
"""
from __future__ import annotations

import numpy as np
import torch

from ..framework import core as _core
from ..framework.core import (Tensor, Parameter, CPUPlace, CUDAPlace, CUDAPinnedPlace, XPUPlace, NPUPlace,  # noqa: F401
                              MLUPlace, IPUPlace, CustomPlace, Place, _wrap)
from ..static.program import Scope, global_scope  # noqa: F401

_Scope = Scope


class _Shape(list):
    """list that is also callable, so ``t.shape`` (2.x) and ``t.shape()`` (pybind LoDTensor) agree"""

    def __call__(self):
        return list(self)


def _offsets_from_lengths(lengths):
    off = [0]
    for n in lengths:
        off.append(off[-1] + int(n))
    return off


def _lengths_from_offsets(off):
    return [int(b) - int(a) for a, b in zip(off[:-1], off[1:])]


class LoDTensor(Tensor):
    """Tensor with a LoD offset table (one list of offsets per level)."""

    def __init__(self, data=None, lod=None):
        super().__init__(data if data is not None else torch.empty(0))
        self._lod = [list(map(int, l)) for l in lod] if lod else []

    @property
    def shape(self):
        return _Shape(list(self._t.shape))

    def set(self, array, place=None):
        dev = _core._to_torch_device(place) if place is not None else torch.device("cpu")
        arr = array.numpy() if isinstance(array, Tensor) else np.asarray(array)
        self._t = torch.from_numpy(np.ascontiguousarray(arr)).to(dev)

    def lod(self):
        return [list(l) for l in self._lod]

    def set_lod(self, lod):
        self._lod = [list(map(int, l)) for l in lod]

    def recursive_sequence_lengths(self):
        return [_lengths_from_offsets(l) for l in self._lod]

    def set_recursive_sequence_lengths(self, lengths):
        self._lod = [_offsets_from_lengths(l) for l in lengths]

    def has_valid_recursive_sequence_lengths(self):
        if not self._lod:
            return True
        n = self._t.shape[0] if self._t.dim() else 0
        for i, off in enumerate(self._lod):
            if off[0] != 0 or any(b < a for a, b in zip(off[:-1], off[1:])):
                return False
            nxt = (len(self._lod[i + 1]) - 1) if i + 1 < len(self._lod) else n
            if off[-1] != nxt:
                return False
        return True

    def _dtype(self):
        return self._t.dtype

    def __array__(self, dtype=None, copy=None):
        a = self._t.detach().cpu().numpy()
        return a.astype(dtype) if dtype is not None else a


class LoDTensorArray(list):
    """``core.LoDTensorArray``: a Python list of tensors (array_write / array_read operate on it)."""

    def append(self, t):
        super().append(t)


def lod_of(x):
    return getattr(x, "_lod", None) or []


def set_lod(x, lod):
    x._lod = [list(map(int, l)) for l in lod]
    return x


class VarDesc:
    class VarType:
        BOOL, INT16, INT32, INT64, FP16, FP32, FP64 = 0, 1, 2, 3, 4, 5, 6
        LOD_TENSOR, SELECTED_ROWS, FEED_MINIBATCH, FETCH_LIST = 7, 8, 9, 10
        STEP_SCOPES, LOD_RANK_TABLE, LOD_TENSOR_ARRAY, PLACE_LIST, READER = 11, 12, 13, 14, 15
        RAW, TUPLE = 17, 18
        SIZE_T, UINT8, INT8, BF16, COMPLEX64, COMPLEX128 = 19, 20, 21, 22, 23, 24


_VT = VarDesc.VarType
_TORCH_OF = {_VT.BOOL: torch.bool, _VT.INT16: torch.int16, _VT.INT32: torch.int32, _VT.INT64: torch.int64,
             _VT.FP16: torch.float16, _VT.FP32: torch.float32, _VT.FP64: torch.float64, _VT.UINT8: torch.uint8,
             _VT.INT8: torch.int8, _VT.BF16: torch.bfloat16, _VT.COMPLEX64: torch.complex64,
             _VT.COMPLEX128: torch.complex128}


def convert_dtype(d):
    """fluid dtype spellings (VarType enum, numpy, str) -> torch dtype"""
    if isinstance(d, int) and not isinstance(d, bool) and d in _TORCH_OF:
        return _TORCH_OF[d]
    return _core.convert_dtype(d)


def is_compiled_with_cuda():
    return False


def is_compiled_with_rocm():
    return True


def is_compiled_with_xpu():
    return False


def is_compiled_with_npu():
    return False


def is_compiled_with_mkldnn():
    return False


def get_cuda_device_count():
    return torch.cuda.device_count()


def _cuda_synchronize(place=None):
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def globals():
    from ..framework import flags
    return flags._FLAGS if hasattr(flags, "_FLAGS") else {}


class EOFException(Exception):
    """raised by Executor.run when a started py_reader has no more batches"""


def CostModel():   # noqa: N802 (the reference's core.CostModel class)
    from ..cost_model import _CoreCostModel
    return _CoreCostModel()


VarBase = Tensor   # the 1.x dygraph tensor class (reference: core.VarBase)
