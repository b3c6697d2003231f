"""Core runtime objects: dtypes, places, the eager ``Tensor`` and ``Parameter``.

Design (MI355X-first): a ``Tensor`` is a thin Python
handle around a ``torch.Tensor`` whose storage lives in HIP device memory (or
host memory for ``CPUPlace``). PyTorch-ROCm supplies storage, the caching
allocator and the autograd tape; the phi-style hot kernels are our own HIP
code (``paddle_hackathon_amd.ops``). The handle carries Paddle semantics:
``stop_gradient`` (default True), ``shape`` as a list, ``place``, ``name`` and
``persistable``.

Reference parity:
  * Tensor methods / operators: python/paddle/fluid/dygraph/varbase_patch_methods.py,
    python/paddle/fluid/dygraph/math_op_patch.py
  * Parameter: python/paddle/fluid/framework.py (EagerParamBase / ParamBase)
  * dtypes: python/paddle/framework/dtype.py
"""
from __future__ import annotations

import itertools
import threading

import numpy as np
import torch

# ----------------------------------------------------------------------------
# dtypes
# ----------------------------------------------------------------------------
bool_ = torch.bool
uint8 = torch.uint8
int8 = torch.int8
int16 = torch.int16
int32 = torch.int32
int64 = torch.int64
float16 = torch.float16
bfloat16 = torch.bfloat16
float32 = torch.float32
float64 = torch.float64
complex64 = torch.complex64
complex128 = torch.complex128
dtype = torch.dtype

_STR2DTYPE = {
    "bool": torch.bool, "uint8": torch.uint8, "int8": torch.int8,
    "int16": torch.int16, "int32": torch.int32, "int64": torch.int64,
    "float16": torch.float16, "fp16": torch.float16, "half": torch.float16,
    "bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "uint16": torch.bfloat16,
    "float32": torch.float32, "fp32": torch.float32, "float": torch.float32,
    "float64": torch.float64, "fp64": torch.float64, "double": torch.float64,
    "complex64": torch.complex64, "complex128": torch.complex128,
    "int": torch.int64, "long": torch.int64,
}
_DTYPE2STR = {
    torch.bool: "bool", torch.uint8: "uint8", torch.int8: "int8",
    torch.int16: "int16", torch.int32: "int32", torch.int64: "int64",
    torch.float16: "float16", torch.bfloat16: "bfloat16",
    torch.float32: "float32", torch.float64: "float64",
    torch.complex64: "complex64", torch.complex128: "complex128",
}

_default_dtype = torch.float32


def convert_dtype(d):
    """Normalise a paddle dtype spec (str / np.dtype / torch.dtype) to torch.dtype."""
    if d is None:
        return None
    if isinstance(d, torch.dtype):
        return d
    if isinstance(d, str):
        try:
            return _STR2DTYPE[d]
        except KeyError:
            raise TypeError(f"unsupported dtype {d!r}")
    if d is bool:
        return torch.bool
    if d is int:
        return torch.int64
    if d is float:
        return _default_dtype
    try:
        npd = np.dtype(d)
    except TypeError:
        raise TypeError(f"unsupported dtype {d!r}")
    if npd == np.dtype("uint16"):  # paddle's bf16 storage convention
        return torch.bfloat16
    return _STR2DTYPE[npd.name]


def dtype_to_str(d):
    return _DTYPE2STR[convert_dtype(d)]


def set_default_dtype(d):
    global _default_dtype
    d = convert_dtype(d)
    if d not in (torch.float16, torch.bfloat16, torch.float32, torch.float64):
        raise TypeError("set_default_dtype only supports floating dtypes")
    _default_dtype = d


def get_default_dtype():
    return _DTYPE2STR[_default_dtype]


def is_floating_dtype(d):
    return d in (torch.float16, torch.bfloat16, torch.float32, torch.float64)


# ----------------------------------------------------------------------------
# places
# ----------------------------------------------------------------------------
class Place:
    """Device placement. ``gpu:N`` is HIP device N (MI355X)."""

    __slots__ = ("_dev",)

    def __init__(self, dev):
        self._dev = torch.device(dev)

    def is_cpu_place(self):
        return self._dev.type == "cpu"

    def is_gpu_place(self):
        return self._dev.type == "cuda"

    def is_cuda_pinned_place(self):
        return False

    def gpu_device_id(self):
        return self._dev.index or 0

    def get_device_id(self):
        return self._dev.index or 0

    @property
    def torch_device(self):
        return self._dev

    def __eq__(self, other):
        return isinstance(other, Place) and self._dev == other._dev

    def __hash__(self):
        return hash(self._dev)

    def __repr__(self):
        if self._dev.type == "cpu":
            return "Place(cpu)"
        return f"Place(gpu:{self._dev.index or 0})"


class CPUPlace(Place):
    __slots__ = ()

    def __init__(self):
        super().__init__("cpu")


class CUDAPlace(Place):
    __slots__ = ()

    def __init__(self, device_id=0):
        super().__init__(f"cuda:{int(device_id)}")


class CUDAPinnedPlace(Place):
    __slots__ = ()

    def __init__(self):
        super().__init__("cpu")

    def is_cuda_pinned_place(self):
        return True


class _OtherVendorPlace(Place):
    """XPU/NPU/MLU/IPU places exist for API compatibility only."""

    __slots__ = ()

    def __init__(self, *a, **k):
        raise RuntimeError(f"{type(self).__name__} is not available in the MI355X framework")


class XPUPlace(_OtherVendorPlace):
    __slots__ = ()


class NPUPlace(_OtherVendorPlace):
    __slots__ = ()


class MLUPlace(_OtherVendorPlace):
    __slots__ = ()


class IPUPlace(_OtherVendorPlace):
    __slots__ = ()


class CustomPlace(_OtherVendorPlace):
    __slots__ = ()


_state = threading.local()
_default_device = None


def _gpu_available():
    return torch.cuda.is_available()


def default_device():
    global _default_device
    if _default_device is None:
        _default_device = torch.device("cuda", torch.cuda.current_device()) if _gpu_available() else torch.device("cpu")
    return _default_device


def set_device(device):
    """paddle.set_device('gpu'|'gpu:N'|'cpu')."""
    global _default_device
    if isinstance(device, Place):
        _default_device = device.torch_device
        if _default_device.type == "cuda":
            torch.cuda.set_device(_default_device)
        return device
    device = str(device).lower()
    if device == "cpu":
        _default_device = torch.device("cpu")
        return CPUPlace()
    if device.startswith("gpu") or device.startswith("cuda") or device.startswith("rocm"):
        if not _gpu_available():
            raise ValueError("The device should not be 'gpu', since PaddlePaddle-AMD is running without a visible MI355X")
        idx = int(device.split(":")[1]) if ":" in device else torch.cuda.current_device()
        torch.cuda.set_device(idx)
        _default_device = torch.device("cuda", idx)
        return CUDAPlace(idx)
    raise ValueError(f"unsupported device {device!r}")


def get_device():
    d = default_device()
    return "cpu" if d.type == "cpu" else f"gpu:{d.index or 0}"


def _to_torch_device(place):
    if place is None:
        return default_device()
    if isinstance(place, Place):
        return place.torch_device
    if isinstance(place, torch.device):
        return place
    s = str(place).lower()
    if s == "cpu":
        return torch.device("cpu")
    if s.startswith("gpu"):
        return torch.device("cuda", int(s.split(":")[1]) if ":" in s else 0)
    return torch.device(s)


def place_of(t: torch.Tensor) -> Place:
    if t.device.type == "cuda":
        return CUDAPlace(t.device.index or 0)
    return CPUPlace()


# ----------------------------------------------------------------------------
# static / dynamic mode flag (static graph recording lives in ../static)
# ----------------------------------------------------------------------------
class _Mode:
    static = False
    trace = False  # op/layer host tracing on (paddle.profiler)
    check_nan_inf = False  # FLAGS_check_nan_inf: scan every op/layer output (and its grad)
    _tl = threading.local()

    # per thread: the dataset trainer's worker threads interpret Programs concurrently
    @property
    def record_depth(self):
        return getattr(self._tl, "d", 0)

    @record_depth.setter
    def record_depth(self, v):
        self._tl.d = v


_mode = _Mode()


def in_dynamic_mode():
    return not _mode.static


# ----------------------------------------------------------------------------
# Tensor
# ----------------------------------------------------------------------------
_name_counter = itertools.count()


def _unique_name(prefix):
    return f"{prefix}_{next(_name_counter)}"


_PRINT_OPTS = {}


def set_printoptions(precision=None, threshold=None, edgeitems=None, sci_mode=None, linewidth=None):
    """paddle.set_printoptions (reference: python/paddle/tensor/to_string.py)."""
    for k, v in (("precision", precision), ("threshold", threshold), ("edgeitems", edgeitems),
                 ("max_line_width", linewidth)):
        if v is not None:
            _PRINT_OPTS[k] = int(v)
    if sci_mode is not None:
        _PRINT_OPTS["floatmode"] = "maxprec"
        _PRINT_OPTS["suppress_small"] = not sci_mode
    torch.set_printoptions(precision=precision, threshold=threshold, edgeitems=edgeitems, linewidth=linewidth,
                           sci_mode=sci_mode)


class Tensor:
    """Eager tensor handle (``paddle.Tensor``)."""

    __slots__ = ("_t", "_name", "_persistable", "__weakref__", "__dict__")
    __array_priority__ = 1000  # numpy defers binary ops to us

    def __init__(self, data=None, dtype=None, place=None, stop_gradient=True, name=None):
        if data is None:
            t = torch.empty(0)
        elif isinstance(data, Tensor):
            t = data._t
        elif isinstance(data, torch.Tensor):
            t = data
        else:
            t = _to_torch(data, dtype, place)
        if dtype is not None:
            t = t.to(convert_dtype(dtype))
        self._t = t
        self._name = name
        self._persistable = False
        if not stop_gradient:
            self.stop_gradient = False

    # -- identity / metadata -------------------------------------------------
    @property
    def name(self):
        if self._name is None:
            self._name = _unique_name("generated_tensor")
        return self._name

    @name.setter
    def name(self, v):
        self._name = v

    @property
    def persistable(self):
        return self._persistable

    @persistable.setter
    def persistable(self, v):
        self._persistable = bool(v)

    @property
    def shape(self):
        # the reference has no 0-d tensors: a full reduction / scalar reads as shape [1]
        return list(self._t.shape) or [1]

    @property
    def ndim(self):
        return self._t.dim()

    def dim(self):
        return self._t.dim()

    ndimension = dim

    @property
    def size(self):
        return self._t.numel()

    def numel(self):
        return self._t.numel()

    @property
    def dtype(self):
        return self._t.dtype

    @property
    def place(self):
        return place_of(self._t)

    @property
    def is_leaf(self):
        return self._t.is_leaf

    @property
    def type(self):
        return "DENSE_TENSOR"

    def is_dense(self):
        return not self._t.is_sparse

    def is_sparse(self):
        return self._t.is_sparse or self._t.layout == torch.sparse_csr

    def is_sparse_coo(self):
        return self._t.is_sparse

    def is_sparse_csr(self):
        return self._t.layout == torch.sparse_csr

    # -- sparse accessors (reference: fluid/dygraph/varbase_patch_methods.py:898-990) -----
    def values(self):
        t = self._t
        if t.layout == torch.sparse_coo:
            return _wrap((t if t.is_coalesced() else t.coalesce()).values())
        return _wrap(t.values() if t.layout == torch.sparse_csr else t)

    def indices(self):
        if not self._t.is_sparse:
            raise ValueError("indices() is only defined for sparse COO tensors")
        return _wrap(self._t.coalesce().indices() if not self._t.is_coalesced() else self._t.indices())

    def crows(self):
        return _wrap(self._t.crow_indices())

    def cols(self):
        return _wrap(self._t.col_indices())

    def nnz(self):
        return self._t._nnz()

    def to_dense(self):
        return _wrap(self._t.to_dense()) if self.is_sparse() else self

    def to_sparse_coo(self, sparse_dim):
        t = self._t.to_dense() if self._t.layout == torch.sparse_csr else self._t
        return _wrap(t.to_sparse(sparse_dim))

    def to_sparse_csr(self):
        t = self._t
        if t.is_sparse:
            t = t.to_dense()
        return _wrap(t.to_sparse_csr())

    # -- autograd ---------------------------------------------------------------
    @property
    def stop_gradient(self):
        return not self._t.requires_grad

    @stop_gradient.setter
    def stop_gradient(self, v):
        v = bool(v)
        if v:
            if self._t.requires_grad:
                self._t = self._t.detach() if not self._t.is_leaf else self._t.requires_grad_(False)
        else:
            if not self._t.requires_grad:
                if not (self._t.is_floating_point() or self._t.is_complex()):
                    return  # integer tensors cannot require grad; paddle silently keeps them constant
                if not self._t.is_leaf:
                    self._t = self._t.detach()
                self._t.requires_grad_(True)

    @property
    def grad(self):
        g = self._t.grad
        return None if g is None else _wrap(g)

    @grad.setter
    def grad(self, v):
        self._t.grad = None if v is None else _unwrap(v)

    def gradient(self):
        g = self._t.grad
        return None if g is None else g.detach().cpu().numpy()

    def backward(self, grad_tensor=None, retain_graph=False):
        from ..autograd import backward as _bw
        _bw([self], None if grad_tensor is None else [grad_tensor], retain_graph)

    def clear_grad(self, set_to_zero=True):
        if self._t.grad is not None:
            if set_to_zero:
                self._t.grad.zero_()
            else:
                self._t.grad = None

    clear_gradient = clear_grad

    def _clear_grad(self):
        self._t.grad = None

    def detach(self):
        return _wrap(self._t.detach())

    def detach_(self):
        self._t = self._t.detach()
        return self

    def register_hook(self, hook):
        def _h(g):
            r = hook(_wrap(g))
            return None if r is None else _unwrap(r)

        handle = self._t.register_hook(_h)
        return handle

    # -- conversion ------------------------------------------------------------
    def numpy(self):
        t = self._t.detach()
        if t.dtype == torch.bfloat16:
            # paddle exposes bf16 as uint16 bit patterns
            a = t.cpu().view(torch.int16).numpy().view(np.uint16)
        else:
            a = t.cpu().numpy()
        # the reference has no 0-d tensors: scalars come back as shape-(1,) arrays (``loss.numpy()[0]``)
        return a.reshape(1) if a.ndim == 0 else a

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a if dtype is None else a.astype(dtype)

    def item(self, *args):
        t = self._t
        if args:
            t = t[args] if len(args) > 1 else t.reshape(-1)[args[0]]
        return t.item()

    def tolist(self):
        return self._t.detach().cpu().tolist()

    def astype(self, dtype):
        return _wrap(self._t.to(convert_dtype(dtype)))

    def cast(self, dtype):
        return self.astype(dtype)

    def cpu(self):
        return _wrap(self._t.cpu())

    def cuda(self, device_id=None, blocking=True):
        dev = torch.device("cuda", device_id if device_id is not None else torch.cuda.current_device())
        return _wrap(self._t.to(dev, non_blocking=not blocking))

    def pin_memory(self):
        return _wrap(self._t.pin_memory())

    def _copy_to(self, place, blocking=True):
        return _wrap(self._t.to(_to_torch_device(place), non_blocking=not blocking))

    def to(self, *args, **kwargs):
        dev = None
        dt = None
        blocking = kwargs.pop("blocking", True)
        for a in list(args) + list(kwargs.values()):
            if isinstance(a, (Place, torch.device)) or (isinstance(a, str) and (a.startswith("gpu") or a.startswith("cpu") or a.startswith("cuda"))):
                dev = _to_torch_device(a)
            elif a is not None:
                dt = convert_dtype(a)
        t = self._t
        if dev is not None:
            t = t.to(dev, non_blocking=not blocking)
        if dt is not None:
            t = t.to(dt)
        return _wrap(t)

    def clone(self):
        return _wrap(self._t.clone())

    def copy_(self, other, blocking=True):
        with torch.no_grad():
            self._t.copy_(_unwrap(other))
        return self

    def set_value(self, value):
        v = value._t if isinstance(value, Tensor) else torch.as_tensor(np.asarray(value))
        with torch.no_grad():
            if list(v.shape) != list(self._t.shape):
                raise ValueError(f"set_value shape mismatch {list(v.shape)} vs {self.shape}")
            self._t.copy_(v.to(self._t.dtype))
        return self

    def get_tensor(self):
        return self

    def value(self):
        return self

    def _is_initialized(self):
        return True

    def is_contiguous(self):
        return self._t.is_contiguous()

    def contiguous(self):
        return _wrap(self._t.contiguous())

    def data_ptr(self):
        return self._t.data_ptr()

    def element_size(self):
        return self._t.element_size()

    @property
    def data(self):
        return _wrap(self._t.detach())

    @data.setter
    def data(self, v):
        with torch.no_grad():
            self._t.data = _unwrap(v)

    # -- python protocol ---------------------------------------------------------
    def __len__(self):
        return self._t.shape[0] if self._t.dim() else 0

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]

    def __bool__(self):
        return bool(self._t)

    def __float__(self):
        return float(self._t.detach())

    def __int__(self):
        return int(self._t.detach())

    def __index__(self):
        return int(self._t)

    def __complex__(self):
        return complex(self._t)

    def __hash__(self):
        return id(self)

    def __repr__(self):
        t = self._t.detach()
        body = np.array2string(self.numpy() if t.dtype != torch.bfloat16 else t.float().cpu().numpy(),
                               separator=", ", prefix="       ", **_PRINT_OPTS)
        return (f"Tensor(shape={self.shape}, dtype={dtype_to_str(t.dtype)}, place={self.place}, "
                f"stop_gradient={self.stop_gradient},\n       {body})")

    __str__ = __repr__

    def __deepcopy__(self, memo):
        cls = type(self)
        o = cls.__new__(cls)
        o._t = self._t.detach().clone().requires_grad_(self._t.requires_grad)
        o._name = self._name
        o._persistable = self._persistable
        if hasattr(self, "__dict__"):
            import copy as _copy
            for k, v in self.__dict__.items():
                setattr(o, k, _copy.deepcopy(v, memo))
        memo[id(self)] = o
        return o

    def __reduce_ex__(self, proto):
        return (_rebuild_tensor, (self.numpy() if self._t.dtype != torch.bfloat16 else self._t.detach().float().cpu().numpy(),
                                  dtype_to_str(self._t.dtype), self.stop_gradient))


def _rebuild_tensor(arr, dt, stop_gradient):
    t = torch.from_numpy(np.asarray(arr)).to(convert_dtype(dt))
    out = _wrap(t.to(default_device()))
    out.stop_gradient = stop_gradient
    return out


class Parameter(Tensor):
    """Trainable parameter (``EagerParamBase``). Always a leaf; persistable."""

    __slots__ = ()

    def __init__(self, shape=None, dtype="float32", data=None, name=None, trainable=True, **kwargs):
        if data is None:
            data = torch.empty([int(s) for s in shape], dtype=convert_dtype(dtype), device=default_device())
        elif isinstance(data, Tensor):
            data = data._t
        data = data.detach()
        self._t = data
        if name is None:   # reference ParamBase: unique_name.generate("_param_base")
            from ..utils import unique_name
            name = unique_name.generate("_param_base")
        self._name = name
        self._persistable = True
        self.optimize_attr = kwargs.get("optimize_attr", {"learning_rate": 1.0})
        self.regularizer = kwargs.get("regularizer", None)
        self.do_model_average = kwargs.get("do_model_average", None)
        self.need_clip = kwargs.get("need_clip", True)
        self.is_distributed = kwargs.get("is_distributed", False)
        self.stop_gradient = not trainable

    @property
    def trainable(self):
        return not self.stop_gradient

    @trainable.setter
    def trainable(self, v):
        self.stop_gradient = not v

    def __repr__(self):
        return "Parameter containing:\n" + super().__repr__()


ParamBase = Parameter
EagerParamBase = Parameter
VarBase = Tensor


# ----------------------------------------------------------------------------
# wrap / unwrap helpers (hot path — keep tiny)
# ----------------------------------------------------------------------------
def _wrap(t):
    o = Tensor.__new__(Tensor)
    o._t = t
    o._name = None
    o._persistable = False
    return o


def _unwrap(x):
    if isinstance(x, Tensor):
        return x._t
    return x


def _wrap_any(x):
    if isinstance(x, torch.Tensor):
        return _wrap(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_wrap_any(v) for v in x)
    return x


def _unwrap_any(x):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, (list, tuple)):
        return type(x)(_unwrap_any(v) for v in x)
    if isinstance(x, dict):
        return {k: _unwrap_any(v) for k, v in x.items()}
    return x


def _to_torch(data, dtype=None, place=None):
    """Materialise python/numpy data as a torch tensor on ``place``."""
    dev = _to_torch_device(place)
    dt = convert_dtype(dtype)
    if isinstance(data, Tensor):
        t = data._t
    elif isinstance(data, torch.Tensor):
        t = data
    elif isinstance(data, np.ndarray):
        if data.dtype == np.uint16 and dt in (None, torch.bfloat16):
            t = torch.from_numpy(data.view(np.int16).copy()).view(torch.bfloat16)
        else:
            if data.dtype == np.float64 and dt is None:
                t = torch.from_numpy(np.ascontiguousarray(data))
            else:
                t = torch.from_numpy(np.ascontiguousarray(data))
    elif isinstance(data, (bool, int, float, complex, np.number, np.bool_)):
        if isinstance(data, (bool, np.bool_)):
            t = torch.tensor(bool(data))
        elif isinstance(data, (int, np.integer)):
            t = torch.tensor(int(data), dtype=torch.int64)
        elif isinstance(data, (float, np.floating)):
            t = torch.tensor(float(data), dtype=_default_dtype)
        else:
            t = torch.tensor(data)
    else:
        # nested lists possibly containing Tensors
        if isinstance(data, (list, tuple)) and any(isinstance(v, Tensor) for v in data):
            t = torch.stack([_to_torch(v, dtype, "cpu") for v in data])
        else:
            arr = np.array(data)
            if arr.dtype == np.float64:
                arr = arr.astype(_DTYPE2STR[_default_dtype] if _default_dtype != torch.bfloat16 else "float32")
            if arr.dtype.kind in "US":
                raise TypeError("string tensors are not supported")
            t = torch.from_numpy(arr)
    if dt is not None and t.dtype != dt:
        t = t.to(dt)
    if t.device != dev:
        t = t.to(dev)
    return t


def to_tensor(data, dtype=None, place=None, stop_gradient=True):
    """paddle.to_tensor (python/paddle/tensor/creation.py:272)."""
    if isinstance(data, Tensor):
        t = data._t.detach().clone()
        if dtype is not None:
            t = t.to(convert_dtype(dtype))
        if place is not None:
            t = t.to(_to_torch_device(place))
    else:
        t = _to_torch(data, dtype, place)
        if t.dtype == torch.float64 and dtype is None and not isinstance(data, np.ndarray):
            t = t.to(_default_dtype)
    out = _wrap(t)
    if not stop_gradient:
        out.stop_gradient = False
    return out


def is_tensor(x):
    return isinstance(x, Tensor)
