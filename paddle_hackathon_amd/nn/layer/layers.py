"""``paddle.nn.Layer`` (reference: python/paddle/fluid/dygraph/layers.py).

Parameters are :class:`Parameter` handles whose HIP storage is owned by the
layer; buffers are plain tensors (persistable ones go into ``state_dict``).
State-dict keys use Paddle's structured names (``fc.weight``) so checkpoints
round-trip with the reference's ``.pdparams`` layout.
"""
from __future__ import annotations

import collections
import copy
import itertools
import re
import weakref

import numpy as np
import torch

from ...framework import core as _core
from ...framework.core import Tensor, Parameter, convert_dtype, default_device, _wrap
from ...framework.param_attr import ParamAttr
from ...utils import unique_name

__all__ = ["Layer", "HookRemoveHelper"]


def _create_parameter(shape, dtype=None, attr=None, is_bias=False, default_initializer=None, name=None,
                      helper="create_parameter"):
    """A parameter named as the reference's LayerHelperBase.create_parameter names it
    (python/paddle/fluid/layer_helper_base.py:329): ``{helper}.w_N`` / ``{helper}.b_N`` from the
    global ``unique_name`` generator, where ``helper`` is the owning Layer's full name
    (``linear_0``) or a per-call ``unique_name.generate(op_type)`` (``fc_0``); an explicit
    ``ParamAttr(name=...)`` / ``name`` wins."""
    from .. import initializer as I
    attr = ParamAttr._to_attr(attr)
    if attr is False:
        return None
    dt = convert_dtype(dtype) or _core._default_dtype
    shape = [int(s) for s in shape]
    pname = attr.name or name
    if pname is None:
        if helper == "create_parameter":   # paddle.create_parameter: LayerHelper("create_parameter")
            helper = unique_name.generate(helper)
        pname = unique_name.generate(helper + (".b" if is_bias else ".w"))
    p = Parameter(shape, dt, name=pname, trainable=attr.trainable,
                  optimize_attr={"learning_rate": attr.learning_rate}, regularizer=attr.regularizer,
                  need_clip=attr.need_clip, do_model_average=attr.do_model_average)
    init = attr.initializer
    if init is None:
        if is_bias:
            init = I._global_bias_init or default_initializer or I.Constant(0.0)
        else:
            init = I._global_weight_init or default_initializer or I.XavierUniform()
    init(p)
    if _core._mode.static:   # the startup program re-initialises it for another Scope
        from ...static.program import note_parameter
        note_parameter(p, init)
    return p


class HookRemoveHelper:
    _next_id = itertools.count()

    def __init__(self, hooks):
        self._hooks_ref = weakref.ref(hooks)
        self._hook_id = next(HookRemoveHelper._next_id)

    def remove(self):
        hooks = self._hooks_ref()
        if hooks is not None and self._hook_id in hooks:
            del hooks[self._hook_id]


class Layer:
    """Base class of all layers."""

    def __init__(self, name_scope=None, dtype="float32"):
        self.training = True
        if name_scope is None:
            name_scope = _camel_to_snake(type(self).__name__)
        # reference fluid/dygraph/layers.py:107 — the GLOBAL unique_name generator, so the names of
        # layers and their parameters (linear_0.w_0) match a reference run of the same script
        self._full_name = unique_name.generate(name_scope)
        self._dtype = dtype
        self._parameters = collections.OrderedDict()
        self._buffers = collections.OrderedDict()
        self._non_persistable_buffer_names_set = set()
        self._sub_layers = collections.OrderedDict()
        self._forward_pre_hooks = collections.OrderedDict()
        self._forward_post_hooks = collections.OrderedDict()
        self._casted_by_pure_fp16 = False
        self._loaddict_holder = collections.OrderedDict()

    # -- modes -------------------------------------------------------------------
    def train(self):
        for l in self.sublayers(include_self=True):
            l.training = True
        return self

    def eval(self):
        for l in self.sublayers(include_self=True):
            l.training = False
        return self

    def full_name(self):
        return self._full_name

    # -- creation -------------------------------------------------------------------
    def create_parameter(self, shape, attr=None, dtype=None, is_bias=False, default_initializer=None):
        return _create_parameter(shape, dtype or self._dtype, attr, is_bias, default_initializer,
                                 helper=self._full_name)

    def create_variable(self, name=None, persistable=None, dtype=None):
        t = _wrap(torch.empty(0, dtype=convert_dtype(dtype) or _core._default_dtype, device=default_device()))
        t.name = ".".join([self._full_name, name]) if name else \
            unique_name.generate(self._full_name + "._generated_var")
        t.persistable = bool(persistable)
        return t

    create_tensor = create_variable

    def add_parameter(self, name, parameter):
        if parameter is None:
            self._parameters[name] = None
        elif not isinstance(parameter, Parameter):
            raise TypeError("parameter must be a Parameter")
        else:
            self._parameters[name] = parameter
        object.__setattr__(self, "__dict__", self.__dict__)
        self.__dict__.pop(name, None)
        return parameter

    def add_sublayer(self, name, sublayer):
        self._sub_layers[str(name)] = sublayer
        return sublayer

    def register_buffer(self, name, tensor, persistable=True):
        if tensor is not None and not isinstance(tensor, Tensor):
            raise TypeError("buffer must be a Tensor")
        self.__dict__.pop(name, None)
        self._buffers[name] = tensor
        if persistable:
            self._non_persistable_buffer_names_set.discard(name)
        else:
            self._non_persistable_buffer_names_set.add(name)

    # -- attribute protocol ----------------------------------------------------------
    def __setattr__(self, name, value):
        d = self.__dict__
        if isinstance(value, Parameter):
            params = d.get("_parameters")
            if params is None:
                raise ValueError("super().__init__() must be called before assigning parameters")
            d.pop(name, None)
            self._sub_layers.pop(name, None) if "_sub_layers" in d else None
            params[name] = value
            return
        if isinstance(value, Layer):
            subs = d.get("_sub_layers")
            if subs is None:
                raise ValueError("super().__init__() must be called before assigning sublayers")
            d.pop(name, None)
            subs[name] = value
            return
        params = d.get("_parameters")
        if params is not None and name in params:
            if value is not None and not isinstance(value, Parameter):
                raise TypeError(f"cannot assign {type(value)} to parameter {name}")
            params[name] = value
            return
        subs = d.get("_sub_layers")
        if subs is not None and name in subs:
            subs[name] = value
            return
        bufs = d.get("_buffers")
        if bufs is not None and name in bufs:
            if value is not None and not isinstance(value, Tensor):
                raise TypeError("buffer must be a Tensor")
            bufs[name] = value
            return
        object.__setattr__(self, name, value)

    def __getattr__(self, name):
        d = self.__dict__
        if "_parameters" in d and name in d["_parameters"]:
            return d["_parameters"][name]
        if "_sub_layers" in d and name in d["_sub_layers"]:
            return d["_sub_layers"][name]
        if "_buffers" in d and name in d["_buffers"]:
            return d["_buffers"][name]
        raise AttributeError(f"'{type(self).__name__}' object has no attribute '{name}'")

    def __delattr__(self, name):
        for k in ("_parameters", "_sub_layers", "_buffers"):
            if name in self.__dict__.get(k, {}):
                del self.__dict__[k][name]
                return
        object.__delattr__(self, name)

    def __dir__(self):
        return list(super().__dir__()) + list(self._parameters) + list(self._sub_layers) + list(self._buffers)

    # -- iteration ---------------------------------------------------------------------
    def parameters(self, include_sublayers=True):
        return [p for _, p in self.named_parameters(include_sublayers=include_sublayers)]

    def named_parameters(self, prefix="", include_sublayers=True):
        seen = set()
        layers = self.named_sublayers(prefix=prefix, include_self=True) if include_sublayers else [(prefix, self)]
        for lp, layer in layers:
            for n, p in layer._parameters.items():
                if p is None or id(p) in seen:
                    continue
                seen.add(id(p))
                yield (lp + "." + n if lp else n), p

    def children(self):
        for _, l in self.named_children():
            yield l

    def named_children(self):
        seen = set()
        for n, l in self._sub_layers.items():
            if l is not None and id(l) not in seen:
                seen.add(id(l))
                yield n, l

    def sublayers(self, include_self=False):
        return [l for _, l in self.named_sublayers(include_self=include_self)]

    def named_sublayers(self, prefix="", include_self=False, layers_set=None):
        if layers_set is None:
            layers_set = set()
        if include_self and id(self) not in layers_set:
            layers_set.add(id(self))
            yield prefix, self
        for n, l in self._sub_layers.items():
            if l is None:
                continue
            p = prefix + "." + n if prefix else n
            yield from l.named_sublayers(prefix=p, include_self=True, layers_set=layers_set)

    def buffers(self, include_sublayers=True):
        return [b for _, b in self.named_buffers(include_sublayers=include_sublayers)]

    def named_buffers(self, prefix="", include_sublayers=True):
        seen = set()
        layers = self.named_sublayers(prefix=prefix, include_self=True) if include_sublayers else [(prefix, self)]
        for lp, layer in layers:
            for n, b in layer._buffers.items():
                if b is None or id(b) in seen:
                    continue
                seen.add(id(b))
                yield (lp + "." + n if lp else n), b

    # -- hooks / call -------------------------------------------------------------------
    def register_forward_pre_hook(self, hook):
        h = HookRemoveHelper(self._forward_pre_hooks)
        self._forward_pre_hooks[h._hook_id] = hook
        return h

    def register_forward_post_hook(self, hook):
        h = HookRemoveHelper(self._forward_post_hooks)
        self._forward_post_hooks[h._hook_id] = hook
        return h

    def __call__(self, *inputs, **kwargs):
        if _core._mode.trace or _core._mode.check_nan_inf:
            if _core._mode.trace:
                from ...profiler import _op_range
                with _op_range(type(self).__name__, "Forward"):
                    out = self._call_impl(*inputs, **kwargs)
            else:
                out = self._call_impl(*inputs, **kwargs)
            if _core._mode.check_nan_inf:
                from ...framework.nan_inf import check_outputs
                check_outputs(self.full_name() if hasattr(self, "full_name") else type(self).__name__, out)
            return out
        return self._call_impl(*inputs, **kwargs)

    def _call_impl(self, *inputs, **kwargs):
        if self._forward_pre_hooks:
            for hook in list(self._forward_pre_hooks.values()):
                r = hook(self, inputs)
                if r is not None:
                    inputs = r if isinstance(r, tuple) else (r,)
        out = self.forward(*inputs, **kwargs)
        if self._forward_post_hooks:
            for hook in list(self._forward_post_hooks.values()):
                r = hook(self, inputs, out)
                if r is not None:
                    out = r
        return out

    def forward(self, *inputs, **kwargs):
        raise NotImplementedError

    def backward(self, *inputs):
        raise ValueError("Layer shouldn't implement backward")

    # -- state ------------------------------------------------------------------------
    def state_dict(self, destination=None, include_sublayers=True, structured_name_prefix="", use_hook=True):
        dest = collections.OrderedDict() if destination is None else destination
        for n, p in self._parameters.items():
            if p is not None:
                dest[structured_name_prefix + n] = p
        for n, b in self._buffers.items():
            if b is not None and n not in self._non_persistable_buffer_names_set:
                dest[structured_name_prefix + n] = b
        if include_sublayers:
            for ln, l in self._sub_layers.items():
                if l is not None:
                    l.state_dict(dest, True, structured_name_prefix + ln + ".", use_hook)
        return dest

    to_static_state_dict = state_dict

    def set_state_dict(self, state_dict, use_structured_name=True):
        own = self.state_dict()
        missing, unexpected = [], []
        by_name = {}
        if not use_structured_name:
            by_name = {v.name: k for k, v in own.items()}
        for k, v in state_dict.items():
            key = k if use_structured_name else by_name.get(k, k)
            if key not in own:
                unexpected.append(k)
                continue
            tgt = own[key]
            src = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
            if isinstance(v, np.ndarray) and v.dtype == np.uint16 and tgt.dtype == torch.bfloat16:
                src = torch.from_numpy(v.view(np.int16).copy()).view(torch.bfloat16)
            if list(src.shape) != list(tgt._t.shape):
                raise ValueError(f"{key}: shape {list(src.shape)} != {tgt.shape}")
            with torch.no_grad():
                tgt._t.copy_(src.to(device=tgt._t.device, dtype=tgt._t.dtype))
        for k in own:
            if k not in state_dict and (use_structured_name or own[k].name not in state_dict):
                missing.append(k)
        return missing, unexpected

    set_dict = set_state_dict
    load_dict = set_state_dict

    # -- conversions -----------------------------------------------------------------------
    def apply(self, fn):
        for l in self.children():
            l.apply(fn)
        fn(self)
        return self

    def _apply_tensors(self, fn, floating_only=True):
        for l in self.sublayers(include_self=True):
            for n, p in list(l._parameters.items()):
                if p is None:
                    continue
                if floating_only and not p._t.is_floating_point():
                    continue
                with torch.no_grad():
                    new = fn(p._t)
                if new is not p._t:
                    rg = p._t.requires_grad
                    p._t = new.detach().requires_grad_(rg)
            for n, b in list(l._buffers.items()):
                if b is None:
                    continue
                if floating_only and not b._t.is_floating_point():
                    if fn.__name__ == "_dev":
                        b._t = fn(b._t)
                    continue
                b._t = fn(b._t)
        return self

    def to(self, device=None, dtype=None, blocking=None):
        dev = _core._to_torch_device(device) if device is not None else None
        dt = convert_dtype(dtype)
        if dev is not None:
            def _dev(t):
                return t.to(dev)
            self._apply_tensors(_dev, floating_only=False)
        if dt is not None:
            self._apply_tensors(lambda t: t.to(dt))
            self._dtype = dt
        return self

    def float(self):
        return self.to(dtype="float32")

    def half(self):
        return self.to(dtype="float16")

    def bfloat16(self):
        return self.to(dtype="bfloat16")

    def clear_gradients(self, set_to_zero=True):
        for p in self.parameters():
            if p.trainable:
                p.clear_grad(set_to_zero)

    def extra_repr(self):
        return ""

    def __repr__(self):
        lines = []
        for n, l in self._sub_layers.items():
            r = repr(l).replace("\n", "\n  ")
            lines.append(f"({n}): {r}")
        main = type(self).__name__ + "(" + self.extra_repr()
        if lines:
            main += "\n  " + "\n  ".join(lines) + "\n"
        return main + ")"

    def __deepcopy__(self, memo):
        cls = type(self)
        o = cls.__new__(cls)
        memo[id(self)] = o
        for k, v in self.__dict__.items():
            object.__setattr__(o, k, copy.deepcopy(v, memo))
        return o

    def _set_name_prefix(self, prefix):
        pass


_FIRST_CAP = re.compile("(.)([A-Z][a-z]+)")
_ALL_CAP = re.compile("([a-z])([A-Z])")


def _camel_to_snake(name):
    """BatchNorm2D -> batch_norm2d, Conv2DTranspose -> conv2d_transpose (the reference's rule)"""
    return _ALL_CAP.sub(r"\1_\2", _FIRST_CAP.sub(r"\1_\2", name)).lower()
