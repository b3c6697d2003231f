"""``paddle.jit`` (reference: python/paddle/fluid/dygraph/jit.py, dygraph_to_static/*, paddle/fluid/jit).

``to_static`` captures a function/Layer into a static ``Program`` by tracing it once per
input signature (shapes/dtypes, or the given ``InputSpec``s) through the op recorder, then
runs the cached Program on later calls — autograd still flows through parameters, so
training works unchanged. In eval mode without grad, ``build_strategy.use_hip_graph``
(default on for inference) freezes the program into a HIP graph: one graph launch per
call instead of one launch per op. ``jit.save`` writes ``.pdmodel``/``.pdiparams``;
``jit.load`` returns a ``TranslatedLayer`` that runs the saved program.
Data-dependent Python control flow (``if`` / ``while`` / ``for range`` on tensors) is transcribed
from the function's AST into static ``cond`` / ``while`` sub-block ops (jit/dy2static.py).
"""
from __future__ import annotations

import functools
import os

import numpy as np
import torch

from ..framework import core as _core
from ..framework.core import Tensor, Parameter, _wrap
from ..nn.layer.layers import Layer
from ..static.program import (Program, program_guard, data as _data, InputSpec, run_program, CompiledProgram,
                              BuildStrategy, Variable)
from .. import static as _static

__all__ = ["to_static", "not_to_static", "save", "load", "TracedLayer", "TranslatedLayer", "ProgramTranslator",
           "set_code_level", "set_verbosity", "StaticFunction", "ignore_module"]

_verbosity = 0
_code_level = 0


def set_verbosity(level=0, also_to_stdout=False):
    global _verbosity
    _verbosity = level


def set_code_level(level=100, also_to_stdout=False):
    global _code_level
    _code_level = level


def ignore_module(modules):
    pass


def _spec_of(x, i):
    if isinstance(x, InputSpec):
        return x
    if isinstance(x, Tensor):
        return InputSpec(x.shape, x.dtype, f"input_{i}")
    if isinstance(x, np.ndarray):
        return InputSpec(list(x.shape), x.dtype, f"input_{i}")
    return None


def _trace(fn, specs, args_template):
    """Trace ``fn`` with static data Variables in place of tensor args; returns (program, in_vars, out)."""
    prog = Program()
    prev = _core._mode.static
    _core._mode.static = True
    try:
        with program_guard(prog, Program()):
            in_vars, call_args = [], []
            k = 0
            for a in args_template:
                if isinstance(a, (Tensor, np.ndarray, InputSpec)):
                    s = specs[k]
                    v = _data(s.name or f"input_{k}", s.shape, s.dtype)
                    v.need_grad = isinstance(a, Tensor) and not a.stop_gradient
                    in_vars.append(v)
                    call_args.append(v)
                    k += 1
                else:
                    call_args.append(a)
            out = fn(*call_args)
    finally:
        _core._mode.static = prev
    return prog, in_vars, out


def _flatten_vars(out):
    if isinstance(out, Variable):
        return [out], lambda vals: vals[0]
    if isinstance(out, (list, tuple)):
        flat, builders = [], []
        for o in out:
            f, b = _flatten_vars(o)
            builders.append((len(flat), len(f), b))
            flat.extend(f)

        def build(vals, _t=type(out)):
            return _t(b(vals[s:s + n]) for s, n, b in builders)
        return flat, build
    if isinstance(out, dict):
        keys = list(out)
        flat, builders = [], []
        for k in keys:
            f, b = _flatten_vars(out[k])
            builders.append((len(flat), len(f), b))
            flat.extend(f)
        return flat, lambda vals: {k: b(vals[s:s + n]) for k, (s, n, b) in zip(keys, builders)}
    return [], lambda vals: out


class _Concrete:
    def __init__(self, prog, in_vars, out):
        self.program = prog
        self.in_vars = in_vars
        self.out_vars, self.build = _flatten_vars(out)
        self.compiled = None

    def __call__(self, tensors, use_graph):
        feed = {v.name: t for v, t in zip(self.in_vars, tensors)}
        if use_graph:
            if self.compiled is None:
                bs = BuildStrategy()
                bs.use_hip_graph = True
                self.compiled = CompiledProgram(self.program, bs)
            vals = self.compiled._run(feed, self.out_vars)
        else:
            vals = run_program(self.program, feed, self.out_vars)
        return self.build(vals)


class StaticFunction:
    def __init__(self, function, input_spec=None, build_strategy=None, layer=None):
        self._fn = function
        self._input_spec = input_spec
        self._build_strategy = build_strategy or BuildStrategy()
        self._layer = layer
        self._cache = {}
        self._enabled = True
        functools.update_wrapper(self, function)

    def __get__(self, instance, owner):
        if instance is None:
            return self
        bound = StaticFunction(self._fn.__get__(instance, owner), self._input_spec, self._build_strategy, instance)
        bound._cache = self._cache
        return bound

    @property
    def dygraph_function(self):
        return self._fn

    def _key(self, args):
        k = []
        for a in args:
            if isinstance(a, Tensor):
                k.append((tuple(a.shape), str(a.dtype), a.stop_gradient))
            elif isinstance(a, np.ndarray):
                k.append((a.shape, str(a.dtype)))
            else:
                k.append(repr(a))
        training = self._layer.training if self._layer is not None else None
        return tuple(k), training, torch.is_grad_enabled()

    @property
    def _static_fn(self):
        """the function with its Python control flow transcribed (jit/dy2static.py)"""
        conv = self.__dict__.get("_conv")
        if conv is None:
            from .dy2static import convert_function
            conv = convert_function(self._fn)
            self.__dict__["_conv"] = conv
        return conv

    def concrete_program_specify_input_spec(self, input_spec=None):
        specs = input_spec or self._input_spec
        prog, in_vars, out = _trace(self._static_fn, specs, specs)
        return _Concrete(prog, in_vars, out)

    def get_concrete_program(self, *args, **kwargs):
        c = self._get(args)
        return c.program, c

    def _get(self, args):
        key = self._key(args)
        c = self._cache.get(key)
        if c is None:
            specs = [s for s in (_spec_of(a, i) for i, a in enumerate(args)) if s is not None]
            if self._input_spec:
                for i, s in enumerate(self._input_spec):
                    if i < len(specs) and isinstance(s, InputSpec):
                        specs[i] = InputSpec(specs[i].shape, specs[i].dtype, s.name or specs[i].name)
            prog, in_vars, out = _trace(self._static_fn, specs, args)
            c = _Concrete(prog, in_vars, out)
            self._cache[key] = c
        return c

    def __call__(self, *args, **kwargs):
        if not self._enabled or not ProgramTranslator.get_instance().enable_to_static or kwargs \
                or not _core.in_dynamic_mode():
            return self._fn(*args, **kwargs)
        c = self._get(args)
        tensors = [a for a in args if isinstance(a, (Tensor, np.ndarray))]
        use_graph = (self._build_strategy.use_hip_graph and not torch.is_grad_enabled()
                     and torch.cuda.is_available() and (self._layer is None or not self._layer.training))
        return c(tensors, use_graph)

    @property
    def concrete_program(self):
        return next(iter(self._cache.values())) if self._cache else None

    def rollback(self):
        return self._fn


def to_static(function=None, input_spec=None, build_strategy=None, property=False):
    def deco(fn):
        if isinstance(fn, Layer):
            layer = fn
            sf = StaticFunction(layer.forward, input_spec, build_strategy, layer)
            object.__setattr__(layer, "forward", sf)
            layer._static_function = sf
            return layer
        return StaticFunction(fn, input_spec, build_strategy)
    if function is not None:
        return deco(function)
    return deco


declarative = to_static


def not_to_static(func=None):
    if func is None:
        return not_to_static
    func._not_to_static = True
    return func


class ProgramTranslator:
    _inst = None

    def __init__(self):
        self.enable_to_static = True

    @classmethod
    def get_instance(cls):
        if cls._inst is None:
            cls._inst = cls()
        return cls._inst

    def enable(self, enable_to_static):
        self.enable_to_static = bool(enable_to_static)

    def get_output(self, dygraph_func, *args, **kwargs):
        return dygraph_func(*args, **kwargs)

    def get_program(self, dygraph_func, *args, **kwargs):
        sf = dygraph_func if isinstance(dygraph_func, StaticFunction) else StaticFunction(dygraph_func)
        c = sf._get(args)
        return c.program, c.in_vars, c.out_vars


def save(layer, path, input_spec=None, **configs):
    """Trace ``layer`` (eval mode) with ``input_spec`` and write ``path.pdmodel`` + ``path.pdiparams``."""
    fn = layer.forward
    if isinstance(fn, StaticFunction):
        spec = input_spec or fn._input_spec
        fn = fn._static_fn
    else:
        from .dy2static import convert_function
        fn = convert_function(fn)
        spec = input_spec
    if spec is None:
        raise ValueError("jit.save needs input_spec (or a to_static layer with input_spec)")
    spec = [s if isinstance(s, InputSpec) else _spec_of(s, i) for i, s in enumerate(spec)]
    for i, s in enumerate(spec):
        if s.name is None:
            s.name = f"input_{i}"
    was_training = getattr(layer, "training", False)
    if isinstance(layer, Layer):
        layer.eval()
    try:
        with torch.no_grad():
            prog, in_vars, out = _trace(fn, spec, spec)
    finally:
        if isinstance(layer, Layer) and was_training:
            layer.train()
    outs, _ = _flatten_vars(out)
    _static.save_inference_model(path, in_vars, outs, None, program=prog)


class TranslatedLayer(Layer):
    def __init__(self, program, feed_names, fetch_vars):
        super().__init__()
        self._program = program
        self._feed_names = feed_names
        self._fetch_vars = fetch_vars
        for p in program.all_parameters():
            self.add_parameter(p.name.replace(".", "_"), p if isinstance(p, Parameter) else Parameter(data=p, name=p.name))

    def forward(self, *inputs):
        feed = dict(zip(self._feed_names, inputs))
        outs = run_program(self._program, feed, self._fetch_vars)
        return outs[0] if len(outs) == 1 else outs

    def program(self, method_name="forward"):
        return self._program


def load(path, **configs):
    """``path.pdmodel`` (ProgramDesc) + ``path.pdiparams`` (save_combine) -> TranslatedLayer whose
    parameters are the loaded persistables marked ``is_parameter``"""
    prog, feeds, fetches = _static.load_inference_model(path)
    return TranslatedLayer(prog, feeds, fetches)


class TracedLayer:
    def __init__(self, program, in_vars, out, layer):
        self._c = _Concrete(program, in_vars, out)
        self._layer = layer
        self.program = program

    @staticmethod
    def trace(layer, inputs):
        inputs = inputs if isinstance(inputs, (list, tuple)) else [inputs]
        specs = [_spec_of(x, i) for i, x in enumerate(inputs)]
        prog, in_vars, out = _trace(layer.forward, specs, inputs)
        tl = TracedLayer(prog, in_vars, out, layer)
        return tl(inputs), tl

    def __call__(self, inputs):
        inputs = inputs if isinstance(inputs, (list, tuple)) else [inputs]
        return self._c(list(inputs), False)

    def set_strategy(self, build_strategy=None, exec_strategy=None):
        pass

    def save_inference_model(self, path, feed=None, fetch=None, **kwargs):
        ins = self._c.in_vars if feed is None else [self._c.in_vars[i] for i in feed]
        outs = self._c.out_vars if fetch is None else [self._c.out_vars[i] for i in fetch]
        _static.save_inference_model(path, ins, outs, None, program=self.program)
