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


class _PyFuncSpec:
    """what a recorded py_func op calls: the user's functions, the outputs' dtypes and which
    inputs / outputs the backward function does not take"""

    def __init__(self, func, backward_func, out_dtypes, skip_x, skip_out):
        self.func, self.backward_func = func, backward_func
        self.out_dtypes, self.skip_x, self.skip_out = out_dtypes, skip_x, skip_out


def _as_lod(t):
    from ..fluid.core import LoDTensor
    v = LoDTensor.__new__(LoDTensor)
    v._t = t.detach()
    v._name = None
    v._persistable = False
    v._lod = []
    return v


class _PyFuncFn(torch.autograd.Function):
    """forward = ``func`` on LoDTensors of the inputs (numpy-convertible), its numpy results
    converted to the declared output dtypes; backward = ``backward_func(x..., out..., dout...)``
    minus the skipped variables, returning one gradient (or None) per input"""

    @staticmethod
    def forward(ctx, spec, *xs):
        ctx.spec = spec
        dev = xs[0].device if xs else _core.default_device()
        res = spec.func(*[_as_lod(x) for x in xs])
        n = len(spec.out_dtypes)
        if n == 0:
            outs = ()
        else:
            res = list(res) if isinstance(res, (list, tuple)) else [res]
            if len(res) != n:
                raise ValueError(f"py_func: func returned {len(res)} value(s) for {n} output variable(s)")
            outs = tuple(_core._to_torch(np.asarray(r._t.cpu() if isinstance(r, Tensor) else r), dtype=dt).to(dev)
                         for r, dt in zip(res, spec.out_dtypes))
        ctx.save_for_backward(*xs, *outs)
        ctx.n_x = len(xs)
        if spec.backward_func is None:
            ctx.mark_non_differentiable(*outs)
        return outs if outs else torch.empty(0, device=dev)

    @staticmethod
    def backward(ctx, *douts):
        spec = ctx.spec
        saved = ctx.saved_tensors
        xs, outs = saved[:ctx.n_x], saved[ctx.n_x:]
        if spec.backward_func is None:
            return (None,) + (None,) * len(xs)
        args = [_as_lod(x) for x, skip in zip(xs, spec.skip_x) if not skip]
        args += [_as_lod(o) for o, skip in zip(outs, spec.skip_out) if not skip]
        args += [None if d is None else _as_lod(d) for d in douts[:len(outs)]]
        res = spec.backward_func(*args)
        res = list(res) if isinstance(res, (list, tuple)) else [res]
        grads = []
        for i, x in enumerate(xs):
            g = res[i] if i < len(res) else None
            if g is None or not x.is_floating_point():
                grads.append(None)
                continue
            g = _core._to_torch(np.asarray(g._t.cpu() if isinstance(g, Tensor) else g), dtype=x.dtype).to(x.device)
            grads.append(g.reshape(x.shape))
        return (None,) + tuple(grads)


def _py_func_run(spec, *xs):
    out = _PyFuncFn.apply(spec, *[x._t for x in xs])
    if not spec.out_dtypes:
        return ()
    return tuple(_wrap(t) for t in (out if isinstance(out, tuple) else (out,)))


def py_func(func, x, out, backward_func=None, skip_vars_in_backward_input=None):
    """A Python operator (reference fluid/layers/nn.py:14140, test_py_func_op.py): ``func`` runs at
    run time on the LoDTensors of ``x`` and its numpy results become the pre-created ``out``
    variables (their dtypes are kept); ``backward_func(x..., out..., dout...)`` — the variables of
    ``skip_vars_in_backward_input`` left out — is the op's gradient. In a static Program this
    records ONE op whose outputs ARE the ``out`` variables (no build-time call of ``func``);
    in dygraph it runs at once. Returns ``out``."""
    xs = [] if x is None else list(x) if isinstance(x, (list, tuple)) else [x]
    outs = [] if out is None else list(out) if isinstance(out, (list, tuple)) else [out]
    for v in xs:
        if not isinstance(v, Tensor):
            raise TypeError("py_func: x must be Variable / list(Variable) / tuple(Variable)")
    skip = [] if skip_vars_in_backward_input is None else list(skip_vars_in_backward_input) \
        if isinstance(skip_vars_in_backward_input, (list, tuple)) else [skip_vars_in_backward_input]
    for v in skip:
        if not any(v is t for t in xs + outs):
            raise ValueError("py_func: skip_vars_in_backward_input must belong to x or out")
    spec = _PyFuncSpec(func, backward_func, [o._t.dtype for o in outs],
                       [any(v is t for v in skip) for t in xs], [any(v is t for v in skip) for t in outs])
    from .program import Variable, OpDesc, default_main_program
    if _core._mode.static and (any(isinstance(v, Variable) for v in xs) or all(isinstance(o, Variable) for o in outs)):
        blk = default_main_program().current_block()
        op = OpDesc("paddle_hackathon_amd.static._py_func_run", _py_func_run, (spec, *xs), {}, tuple(outs))
        for o in outs:
            o.op = op
            if isinstance(o, Variable):
                o.stop_gradient = backward_func is None
        blk.append_op(op)
    else:
        res = _py_func_run(spec, *xs)
        for o, r in zip(outs, res):
            o._t = r._t
    if out is None:
        return None
    return out if isinstance(out, (list, tuple)) else outs[0]


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
