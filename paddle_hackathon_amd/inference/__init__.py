"""``paddle.inference`` — deployment predictor (reference: paddle/fluid/inference/api/
analysis_predictor.cc, paddle_analysis_config.h, python/paddle/fluid/inference/wrapper.py).

A Predictor loads a saved inference program (``jit.save`` / ``static.save_inference_model``
format: a framework.proto ProgramDesc + save_combine params), runs the IR pass pipeline over it
(``Config.switch_ir_optim``, default on; ``Config.pass_builder()`` edits the list — conv+BN
folding, conv+add+ReLU, fc(+act), skip-LayerNorm and multi-head attention fusion, dropout /
identity-scale removal, constant folding, dead-code elimination; inference/passes.py), with
``PrecisionType.Half``/``Bfloat16`` the auto-mixed-precision pass (GEMM/conv weights in 16 bit,
norm parameters fp32, feeds cast on entry), and runs it; on the
MI355X with ``enable_use_gpu`` the whole forward is captured into a HIP graph per input
signature (``Config.enable_hip_graph``, default on) so a request costs one graph launch.
TensorRT / MKLDNN / Lite / XPU switches of the reference are accepted and ignored."""
from __future__ import annotations

import enum
import os

import numpy as np
import torch

from ..framework import core as _core
from ..framework.core import _wrap, convert_dtype

__all__ = ["Config", "DataType", "PlaceType", "PrecisionType", "BackendType", "Tensor", "Predictor",
           "create_predictor", "get_version", "get_trt_compile_version", "convert_to_mixed_precision",
           "get_trt_runtime_version", "get_num_bytes_of_data_type", "PredictorPool"]


class DataType(enum.IntEnum):
    FLOAT32 = 0
    INT64 = 1
    INT32 = 2
    UINT8 = 3
    INT8 = 4
    FLOAT16 = 5
    BFLOAT16 = 6
    BOOL = 7


_DT_NP = {DataType.FLOAT32: np.float32, DataType.INT64: np.int64, DataType.INT32: np.int32, DataType.UINT8: np.uint8,
          DataType.INT8: np.int8, DataType.FLOAT16: np.float16, DataType.BOOL: np.bool_}
_DT_BYTES = {DataType.FLOAT32: 4, DataType.INT64: 8, DataType.INT32: 4, DataType.UINT8: 1, DataType.INT8: 1,
             DataType.FLOAT16: 2, DataType.BFLOAT16: 2, DataType.BOOL: 1}


class PlaceType(enum.IntEnum):
    UNK = -1
    CPU = 0
    GPU = 1
    XPU = 2
    NPU = 3
    IPU = 4
    CUSTOM = 5


class PrecisionType(enum.IntEnum):
    Float32 = 0
    Int8 = 1
    Half = 2
    Bfloat16 = 3


class BackendType(enum.IntEnum):
    CPU = 0
    GPU = 1
    XPU = 2
    NPU = 3


def get_version():
    from .. import __version__
    return f"version: {__version__}\ncommit: mi355x\nbranch: main\nWITH_GPU: ON (HIP/gfx950)\nWITH_TENSORRT: OFF"


def get_trt_compile_version():
    return (0, 0, 0)


def get_trt_runtime_version():
    return (0, 0, 0)


def get_num_bytes_of_data_type(dtype):
    return _DT_BYTES[DataType(dtype)]


class Config:
    def __init__(self, model_dir_or_prog_file=None, params_file=None):
        self._prog_file = self._params_file = self._model_dir = None
        if params_file is not None:
            self._prog_file, self._params_file = model_dir_or_prog_file, params_file
        elif model_dir_or_prog_file is not None:
            self._model_dir = model_dir_or_prog_file
        self._use_gpu = False
        self._device_id = 0
        self._precision = PrecisionType.Float32
        self._hip_graph = True
        self._ir_optim = True
        self._memory_optim = False
        self._cpu_threads = 1
        self._glog = True
        self._pass_builder = None
        self._mp_black_list = set()

    # model location ----------------------------------------------------------------
    def set_model(self, prog_file, params_file=None):
        if params_file is None:
            self._model_dir = prog_file
        else:
            self._prog_file, self._params_file = prog_file, params_file

    def set_prog_file(self, f):
        self._prog_file = f

    def set_params_file(self, f):
        self._params_file = f

    def prog_file(self):
        return self._prog_file

    def params_file(self):
        return self._params_file

    def model_dir(self):
        return self._model_dir

    def _prefix(self):
        if self._prog_file:
            return self._prog_file[:-len(".pdmodel")] if self._prog_file.endswith(".pdmodel") else self._prog_file
        d = self._model_dir
        for cand in ("inference", "model", "__model__"):
            if os.path.exists(os.path.join(d, cand + ".pdmodel")):
                return os.path.join(d, cand)
        files = [f for f in os.listdir(d) if f.endswith(".pdmodel")]
        if not files:
            raise FileNotFoundError(f"no .pdmodel under {d}")
        return os.path.join(d, files[0][:-len(".pdmodel")])

    # device / precision ------------------------------------------------------------
    def enable_use_gpu(self, memory_pool_init_size_mb=100, device_id=0, precision_mode=PrecisionType.Float32):
        self._use_gpu = True
        self._device_id = device_id
        self._precision = PrecisionType(precision_mode)

    def disable_gpu(self):
        self._use_gpu = False

    def use_gpu(self):
        return self._use_gpu

    def gpu_device_id(self):
        return self._device_id

    def enable_hip_graph(self, enable=True):
        self._hip_graph = enable

    def switch_ir_optim(self, x=True):
        self._ir_optim = x

    def ir_optim(self):
        return self._ir_optim

    def pass_builder(self):
        if self._pass_builder is None:
            from .passes import PassStrategy
            self._pass_builder = PassStrategy()
        return self._pass_builder

    def delete_pass(self, name):
        self.pass_builder().delete_pass(name)

    def exp_disable_mixed_precision_ops(self, black_list):
        self._mp_black_list |= set(black_list)

    def enable_memory_optim(self, x=True):
        self._memory_optim = x

    def set_cpu_math_library_num_threads(self, n):
        self._cpu_threads = n
        torch.set_num_threads(n)

    def cpu_math_library_num_threads(self):
        return self._cpu_threads

    def disable_glog_info(self):
        self._glog = False

    def switch_use_feed_fetch_ops(self, x=False):
        pass

    def switch_specify_input_names(self, x=True):
        pass

    # accepted-and-ignored back-ends of other vendors / engines
    def enable_tensorrt_engine(self, *a, **k):
        pass

    def enable_mkldnn(self):
        pass

    def enable_xpu(self, *a, **k):
        pass

    def enable_lite_engine(self, *a, **k):
        pass

    def tensorrt_engine_enabled(self):
        return False

    def summary(self):
        return (f"model: {self._model_dir or self._prog_file}\nuse_gpu: {self._use_gpu} (device {self._device_id})\n"
                f"precision: {self._precision.name}\nhip_graph: {self._hip_graph}\nir_optim: {self._ir_optim}")


class Tensor:
    """Input/output handle (ZeroCopyTensor)."""

    def __init__(self, name, predictor):
        self._name = name
        self._p = predictor
        self._shape = None

    def name(self):
        return self._name

    def reshape(self, shape):
        self._shape = list(shape)

    def copy_from_cpu(self, data):
        a = np.ascontiguousarray(data)
        if self._shape is not None and list(a.shape) != self._shape:
            a = a.reshape(self._shape)
        self._p._inputs[self._name] = a

    def share_external_data(self, data):
        self._p._inputs[self._name] = data

    def copy_to_cpu(self):
        t = self._p._outputs[self._name]
        t = t._t if hasattr(t, "_t") else t
        if t.dtype == torch.bfloat16:
            t = t.float()
        return t.detach().cpu().numpy()

    def shape(self):
        if self._name in self._p._outputs:
            return list(self._p._outputs[self._name].shape)
        if self._name in self._p._inputs:
            return list(np.shape(self._p._inputs[self._name]))
        return self._shape

    def type(self):
        a = self._p._outputs.get(self._name, self._p._inputs.get(self._name))
        dt = str(getattr(a, "dtype", "float32"))
        for k, v in {"float32": DataType.FLOAT32, "int64": DataType.INT64, "int32": DataType.INT32,
                     "float16": DataType.FLOAT16, "bfloat16": DataType.BFLOAT16, "uint8": DataType.UINT8,
                     "int8": DataType.INT8, "bool": DataType.BOOL}.items():
            if k in dt:
                return v
        return DataType.FLOAT32

    def lod(self):
        return []

    def set_lod(self, lod):
        pass


class Predictor:
    def __init__(self, config, _shared=None):
        from .. import static
        self._config = config
        if config.use_gpu() and torch.cuda.is_available():
            torch.cuda.set_device(config.gpu_device_id())
            self._device = torch.device("cuda", config.gpu_device_id())
        else:
            self._device = torch.device("cpu")
        if _shared is not None:
            self._prog, self._feeds, self._fetches = _shared
            self._amp = {PrecisionType.Half: torch.float16,
                         PrecisionType.Bfloat16: torch.bfloat16}.get(config._precision)
            self.ir_stats = {}
        else:
            prev = _core._default_device
            _core._default_device = self._device
            try:
                self._prog, self._feeds, self._fetches = static.load_inference_model(config._prefix())
            finally:
                _core._default_device = prev
            self._fetches = list(self._fetches)
            self._amp = {PrecisionType.Half: torch.float16,
                         PrecisionType.Bfloat16: torch.bfloat16}.get(config._precision)
            self.ir_stats = {}
            if config.ir_optim():
                self.ir_stats = config.pass_builder().run(self._prog, self._fetches, amp_dtype=self._amp,
                                                          black_list=config._mp_black_list)
            elif self._amp is not None:
                self._cast_params(config._precision)
        bs = static.BuildStrategy()
        bs.use_hip_graph = bool(config._hip_graph and self._device.type == "cuda")
        self._compiled = static.CompiledProgram(self._prog, bs)
        self._inputs, self._outputs = {}, {}
        self._fetch_names = [getattr(v, "name", f"fetch_{i}") for i, v in enumerate(self._fetches)]

    def _cast_params(self, precision):
        dt = {PrecisionType.Half: torch.float16, PrecisionType.Bfloat16: torch.bfloat16}.get(precision)
        if dt is None:
            return
        with torch.no_grad():
            for p in self._prog.all_parameters():
                if p._t.is_floating_point():
                    p._t = p._t.to(dt)

    def get_input_names(self):
        return list(self._feeds)

    def get_output_names(self):
        return list(self._fetch_names)

    def get_input_handle(self, name):
        return Tensor(name, self)

    def get_output_handle(self, name):
        return Tensor(name, self)

    def run(self, inputs=None):
        if inputs is not None:
            for n, a in zip(self._feeds, inputs):
                self._inputs[n] = a.copy_to_cpu() if isinstance(a, Tensor) else a
        prev = _core._default_device
        _core._default_device = self._device
        try:
            with torch.no_grad():
                feed = {k: (v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))).to(self._device)
                        for k, v in self._inputs.items()}
                if self._amp is not None:   # low-precision program: float feeds enter in its dtype
                    feed = {k: v.to(self._amp) if v.is_floating_point() else v for k, v in feed.items()}
                outs = self._compiled._run({k: _wrap(v) for k, v in feed.items()}, self._fetches)
        finally:
            _core._default_device = prev
        self._outputs = dict(zip(self._fetch_names, outs))
        if inputs is not None:
            res = []
            for n in self._fetch_names:
                h = Tensor(n, self)
                res.append(h)
            return res
        return True

    def clone(self):
        return Predictor(self._config, _shared=(self._prog, self._feeds, self._fetches))

    def clear_intermediate_tensor(self):
        self._outputs = {}

    def try_shrink_memory(self):
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        return 0


def create_predictor(config):
    return Predictor(config)


class PredictorPool:
    def __init__(self, config, size=1):
        first = Predictor(config)
        self._preds = [first] + [first.clone() for _ in range(size - 1)]

    def retrive(self, idx):
        return self._preds[idx]

    retrieve = retrive


def convert_to_mixed_precision(model_file, params_file, mixed_model_file, mixed_params_file, mixed_precision,
                               backend, keep_io_types=True, black_list=None):
    """Re-save a model with floating weights cast to fp16/bf16 (ops in ``black_list`` keep fp32
    weights)."""
    from .. import static
    prefix = model_file[:-len(".pdmodel")] if model_file.endswith(".pdmodel") else model_file
    prog, feeds, fetches = static.load_inference_model(prefix)
    dt = {PrecisionType.Half: torch.float16, PrecisionType.Bfloat16: torch.bfloat16}[PrecisionType(mixed_precision)]
    black = set(black_list or [])
    keep = set()
    for op in prog.global_block().ops:
        if op.type in black:
            for a in list(op.args) + list(op.kwargs.values()):
                if hasattr(a, "name"):
                    keep.add(a.name)
    with torch.no_grad():
        for p in prog.all_parameters():
            if p._t.is_floating_point() and p.name not in keep:
                p._t = p._t.to(dt)
    out_prefix = mixed_model_file[:-len(".pdmodel")] if mixed_model_file.endswith(".pdmodel") else mixed_model_file
    feed_vars = [prog.global_block().vars[n] for n in feeds]
    static.save_inference_model(out_prefix, feed_vars, fetches, None, program=prog)
    if mixed_params_file and mixed_params_file != out_prefix + ".pdiparams":
        os.replace(out_prefix + ".pdiparams", mixed_params_file)
