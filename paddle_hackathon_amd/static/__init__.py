"""``paddle.static`` (reference: python/paddle/static/__init__.py, static/io.py, fluid/io.py)."""
from __future__ import annotations

import json
import os
import pickle

import numpy as np
import torch

from ..framework import core as _core
from ..framework.core import Tensor, Parameter, _wrap, CPUPlace, CUDAPlace
from ..framework.param_attr import WeightNormParamAttr  # noqa: F401
from ..framework.io import save as _save_obj, load as _load_obj
from .program import (Variable, Program, Block, OpDesc, default_main_program, default_startup_program,  # noqa: F401
                      program_guard, data, Executor, global_scope, scope_guard, append_backward, gradients,
                      enable_static, disable_static, name_scope, CompiledProgram, BuildStrategy, ExecutionStrategy,
                      InputSpec, Scope, run_program, plan_program_memory)
from . import nn  # noqa: F401


__all__ = ["BuildStrategy", "CompiledProgram", "ExecutionStrategy", "Executor", "ExponentialMovingAverage", "InputSpec",
           "IpuCompiledProgram", "IpuStrategy", "ParallelExecutor", "Print", "Program", "Variable",
           "WeightNormParamAttr", "accuracy", "append_backward", "auc", "cpu_places", "create_global_var",
           "create_parameter", "ctr_metric_bundle", "cuda_places", "data", "default_main_program",
           "default_startup_program", "deserialize_persistables", "deserialize_program", "device_guard",
           "exponential_decay", "global_scope", "gradients", "ipu_shard_guard", "load", "load_from_file",
           "load_inference_model", "load_program_state", "mlu_places", "name_scope", "normalize_program", "npu_places",
           "program_guard", "py_func", "save", "save_inference_model", "save_to_file", "scope_guard",
           "serialize_persistables", "serialize_program", "set_ipu_shard", "set_program_state", "xpu_places",
           "enable_static", "disable_static", "nn"]

ParallelExecutor = Executor


def cpu_places(device_count=None):
    return [CPUPlace() for _ in range(device_count or 1)]


def cuda_places(device_ids=None):
    if device_ids is None:
        device_ids = list(range(torch.cuda.device_count())) if torch.cuda.is_available() else []
    return [CUDAPlace(i) for i in device_ids]


def _no_device(kind):
    def f(*a, **k):
        raise RuntimeError(f"{kind} devices are not part of the MI355X build")
    return f


xpu_places = _no_device("XPU")
npu_places = _no_device("NPU")
mlu_places = _no_device("MLU")


class IpuStrategy:
    def __init__(self):
        raise RuntimeError("IPU is not part of the MI355X build")


class IpuCompiledProgram(IpuStrategy):
    pass


def ipu_shard_guard(index=-1, stage=-1):
    raise RuntimeError("IPU is not part of the MI355X build")


set_ipu_shard = ipu_shard_guard


class device_guard:
    """ops recorded inside carry ``op_device`` = ``device`` ("gpu:k" names pipeline stage k for
    the static pipeline pass, parallel/fleet/static_pipeline.py; reference fluid/framework.py
    device_guard)"""

    def __init__(self, device=None):
        self.device = device

    def __enter__(self):
        from .program import _OP_DEVICE
        self.prev = _OP_DEVICE[0]
        _OP_DEVICE[0] = self.device
        return self

    def __exit__(self, *a):
        from .program import _OP_DEVICE
        _OP_DEVICE[0] = self.prev
        return False


def create_parameter(shape, dtype, name=None, attr=None, is_bias=False, default_initializer=None):
    from ..nn.layer.layers import _create_parameter
    return _create_parameter(shape, dtype, attr, is_bias, default_initializer, name=name)


def create_global_var(shape, value, dtype, persistable=False, force_cpu=False, name=None):
    from ..tensor.creation import full
    t = full(shape, value, dtype)
    t.persistable = persistable
    if name:
        t.name = name
    return t


def Print(input, first_n=-1, message=None, summarize=20, print_tensor_name=True, print_tensor_type=True,
          print_tensor_shape=True, print_tensor_lod=True, print_phase="both"):
    """static.Print = fluid.layers.Print (one recorded print op)"""
    from ..fluid.layers.control_flow import Print as _P
    return _P(input, first_n, message, summarize, print_tensor_name, print_tensor_type, print_tensor_shape,
              print_tensor_lod, print_phase)


def py_func(func, x, out, backward_func=None, skip_vars_in_backward_input=None):
    from ..framework.dispatch import static_op
    xs = x if isinstance(x, (list, tuple)) else [x]

    def _call(*vals):
        r = func(*vals)
        return r
    return static_op(_call, "py_func")(*xs)


def accuracy(input, label, k=1, correct=None, total=None):
    from ..metric import accuracy as _acc
    return _acc(input, label, k, correct, total)


def auc(input, label, curve="ROC", num_thresholds=2 ** 12 - 1, topk=1, slide_steps=1, ins_tag_weight=None):
    """static.auc = fluid.layers.auc (persistable stat buffers, two recorded auc ops)"""
    from ..fluid.layers.metric_op import auc as _auc
    return _auc(input, label, curve, num_thresholds, topk, slide_steps)


def ctr_metric_bundle(input, label, ins_tag_weight=None):
    p = input._t.reshape(-1).float()
    y = label._t.reshape(-1).float()
    sq = ((p - y) ** 2).sum()
    ab = (p - y).abs().sum()
    return tuple(_wrap(t) for t in (sq, ab, p.sum(), y.sum(), torch.tensor(float(p.numel())), torch.tensor(float(p.numel()))))


def exponential_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    from ..optimizer.lr import LambdaDecay
    import math
    fn = (lambda e: decay_rate ** math.floor(e / decay_steps)) if staircase else (lambda e: decay_rate ** (e / decay_steps))
    return LambdaDecay(learning_rate, fn)


class ExponentialMovingAverage:
    """EMA of parameters (reference: fluid/optimizer.py:ExponentialMovingAverage)."""

    def __init__(self, decay=0.999, thres_steps=None, name=None):
        self._decay = decay
        self._shadow = {}
        self._backup = {}
        self._step = 0

    def update(self, parameters=None):
        params = parameters if parameters is not None else default_main_program().all_parameters()
        self._step += 1
        d = min(self._decay, (1 + self._step) / (10 + self._step))
        with torch.no_grad():
            for p in params:
                s = self._shadow.get(p.name)
                if s is None:
                    self._shadow[p.name] = (p, p._t.detach().float().clone())
                else:
                    s[1].mul_(d).add_(p._t.float(), alpha=1 - d)

    class _Guard:
        def __init__(self, ema, need_restore):
            self.ema, self.need_restore = ema, need_restore

        def __enter__(self):
            with torch.no_grad():
                for name, (p, s) in self.ema._shadow.items():
                    self.ema._backup[name] = p._t.detach().clone()
                    p._t.copy_(s.to(p._t.dtype))
            return self

        def __exit__(self, *a):
            if self.need_restore:
                self.ema.restore()
            return False

    def apply(self, executor=None, need_restore=True):
        return self._Guard(self, need_restore)

    def restore(self, executor=None):
        with torch.no_grad():
            for name, (p, s) in self._shadow.items():
                if name in self._backup:
                    p._t.copy_(self._backup.pop(name))


# ----------------------------------------------------------------------------- persistence
def _params_of(program):
    return {p.name: p for p in program.all_parameters()}


def save(program, model_path, protocol=4, **configs):
    base = model_path[:-len(".pdparams")] if model_path.endswith(".pdparams") else model_path
    d = os.path.dirname(base)
    if d:
        os.makedirs(d, exist_ok=True)
    _save_obj({k: v for k, v in _params_of(program).items()}, base + ".pdparams", protocol)
    save_to_file(base + ".pdmodel", serialize_program([v for v in program.list_vars() if getattr(v, "is_data", False)],
                                                      [], program=program))


def load(program, model_path, executor=None, var_list=None):
    base = model_path[:-len(".pdparams")] if model_path.endswith(".pdparams") else model_path
    state = _load_obj(base + ".pdparams", return_numpy=True)
    set_program_state(program, state)


def load_program_state(model_path, var_list=None):
    base = model_path[:-len(".pdparams")] if model_path.endswith(".pdparams") else model_path
    return _load_obj(base + ".pdparams", return_numpy=True)


def set_program_state(program, state_dict):
    own = _params_of(program)
    for k, v in state_dict.items():
        if k in own:
            own[k].set_value(np.asarray(v) if not isinstance(v, Tensor) else v.numpy())


def _as_list(v):
    return list(v) if isinstance(v, (list, tuple)) else [v]


def serialize_program(feed_vars, fetch_vars, **kwargs):
    """ProgramDesc bytes (framework.proto wire format; static/serialize.py). ``training=True``: the
    whole training program (reference <type>_grad and optimizer ops, static/ref_train.py), which
    loads back with ``deserialize_program`` + ``deserialize_persistables`` and keeps training"""
    from .serialize import serialize_program_bytes
    program = kwargs.get("program") or default_main_program()
    return serialize_program_bytes(program, _as_list(feed_vars), _as_list(fetch_vars), kwargs.get("training", False))


def serialize_persistables(feed_vars, fetch_vars, executor=None, **kwargs):
    """the persistables the (pruned) program reads, as one save_combine stream sorted by name;
    ``training=True``: those of the whole training program, optimizer accumulators included"""
    from .serialize import serialize_persistables_bytes
    program = kwargs.get("program") or default_main_program()
    return serialize_persistables_bytes(program, _as_list(feed_vars), _as_list(fetch_vars),
                                        kwargs.get("training", False))


def deserialize_program(data):
    from .serialize import parse_program
    return _ProgramStub(parse_program(data))


class _ProgramStub:
    """A deserialised ProgramDesc whose persistable values arrive with deserialize_persistables."""

    def __init__(self, desc):
        self.desc = desc
        self.program = None

    @property
    def num_blocks(self):
        return len(self.desc.blocks)


def deserialize_persistables(program, data, executor=None):
    from .serialize import desc_to_program, load_persistables
    if isinstance(program, _ProgramStub):
        persist = load_persistables(program.desc, data)
        prog, feeds, fetches = desc_to_program(program.desc, persist)
        program.program, program.feeds, program.fetches = prog, feeds, fetches
        return prog
    from .serialize import program_to_desc
    desc, _ = program_to_desc(program, [], [])
    set_program_state(program, {k: v for k, v in load_persistables(desc, data).items()})
    return program


def save_to_file(path, content):
    with open(path, "wb") as f:
        f.write(content)


def load_from_file(path):
    with open(path, "rb") as f:
        return f.read()


def normalize_program(program, feed_vars, fetch_vars):
    return program.clone(for_test=True)


def save_inference_model(path_prefix, feed_vars, fetch_vars, executor=None, **kwargs):
    """Writes ``{prefix}.pdmodel`` (a framework.proto ProgramDesc with feed/fetch ops) and
    ``{prefix}.pdiparams`` (the persistables as one save_combine LoDTensor stream, sorted by name)."""
    program = kwargs.get("program") or default_main_program()
    program = program.clone(for_test=True)
    d = os.path.dirname(path_prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    save_to_file(path_prefix + ".pdmodel", serialize_program(feed_vars, fetch_vars, program=program))
    save_to_file(path_prefix + ".pdiparams", serialize_persistables(feed_vars, fetch_vars, executor, program=program))


def load_inference_model(path_prefix, executor=None, **kwargs):
    stub = deserialize_program(load_from_file(path_prefix + ".pdmodel"))
    prog = deserialize_persistables(stub, load_from_file(path_prefix + ".pdiparams"), executor)
    return [prog, [v.name for v in stub.feeds], stub.fetches]


def __getattr__(name):   # paddle.static.amp: imported on first use (it imports fluid, which imports static)
    if name == "amp":
        import importlib
        return importlib.import_module(".amp", __name__)
    raise AttributeError(name)
