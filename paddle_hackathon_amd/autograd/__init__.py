"""Eager autograd (reference: paddle/fluid/eager/backward.cc,
python/paddle/autograd/{backward_mode.py,py_layer.py}, python/paddle/fluid/dygraph/base.py:grad).

The tape is PyTorch-ROCm's autograd engine; this module gives it Paddle's API:
``backward`` over several roots, ``grad`` with ``no_grad_vars`` /
``allow_unused`` / ``create_graph``, ``PyLayer`` custom ops and grad-mode guards.
"""
from __future__ import annotations

import contextlib
import functools

import torch

from ..framework.core import Tensor, _wrap, _unwrap

__all__ = ["backward", "grad", "PyLayer", "PyLayerContext", "no_grad", "enable_grad",
           "set_grad_enabled", "is_grad_enabled", "functional", "jacobian", "hessian", "vjp", "jvp",
           "saved_tensors_hooks"]


def backward(tensors, grad_tensors=None, retain_graph=False):
    if isinstance(tensors, Tensor):
        tensors = [tensors]
    roots = [t._t for t in tensors]
    grads = None
    if grad_tensors is not None:
        if isinstance(grad_tensors, Tensor):
            grad_tensors = [grad_tensors]
        grads = [None if g is None else _unwrap(g) for g in grad_tensors]
    else:
        grads = [torch.ones_like(r) if r.numel() != 1 or r.dim() else None for r in roots]
    torch.autograd.backward(roots, grads, retain_graph=retain_graph)


def grad(outputs, inputs, grad_outputs=None, retain_graph=None, create_graph=False,
         only_inputs=True, allow_unused=False, no_grad_vars=None):
    single = isinstance(inputs, Tensor)
    outs = [outputs] if isinstance(outputs, Tensor) else list(outputs)
    ins = [inputs] if single else list(inputs)
    gouts = None
    if grad_outputs is not None:
        if isinstance(grad_outputs, Tensor):
            grad_outputs = [grad_outputs]
        gouts = [None if g is None else _unwrap(g) for g in grad_outputs]
    if retain_graph is None:
        retain_graph = create_graph
    if no_grad_vars is not None:
        nv = [no_grad_vars] if isinstance(no_grad_vars, Tensor) else list(no_grad_vars)
        nvid = {id(v._t) for v in nv}
        mask = [id(i._t) not in nvid for i in ins]
    else:
        mask = [True] * len(ins)
    sel = [i._t for i, m in zip(ins, mask) if m]
    res = torch.autograd.grad([o._t for o in outs], sel, gouts, retain_graph=retain_graph,
                              create_graph=create_graph, allow_unused=allow_unused)
    it = iter(res)
    out = [(_wrap(g) if (g := next(it)) is not None else None) if m else None for m in mask]
    return out


no_grad_ = torch.no_grad


class no_grad(contextlib.ContextDecorator):
    """``paddle.no_grad`` — usable as context manager or decorator."""

    def __enter__(self):
        self._prev = torch.is_grad_enabled()
        torch.set_grad_enabled(False)
        return self

    def __exit__(self, *exc):
        torch.set_grad_enabled(self._prev)
        return False


class enable_grad(contextlib.ContextDecorator):
    def __enter__(self):
        self._prev = torch.is_grad_enabled()
        torch.set_grad_enabled(True)
        return self

    def __exit__(self, *exc):
        torch.set_grad_enabled(self._prev)
        return False


class set_grad_enabled(contextlib.ContextDecorator):
    def __init__(self, mode):
        self._mode = bool(mode)
        self._prev = torch.is_grad_enabled()
        torch.set_grad_enabled(self._mode)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        torch.set_grad_enabled(self._prev)
        return False


def is_grad_enabled():
    return torch.is_grad_enabled()


saved_tensors_hooks = torch.autograd.graph.saved_tensors_hooks


# ----------------------------------------------------------------------------
# PyLayer (reference: python/paddle/autograd/py_layer.py)
# ----------------------------------------------------------------------------
class PyLayerContext:
    def __init__(self, tctx):
        self._tctx = tctx
        self.not_inplace_tensors = ()
        self.materialize_grads = True

    def save_for_backward(self, *tensors):
        self._tctx.save_for_backward(*[_unwrap(t) for t in tensors])
        self._saved_kinds = [isinstance(t, Tensor) for t in tensors]

    def saved_tensor(self):
        return tuple(_wrap(t) if t is not None else None for t in self._tctx.saved_tensors)

    def mark_not_inplace(self, *args):
        self.not_inplace_tensors = args

    def mark_non_differentiable(self, *args):
        self._tctx.mark_non_differentiable(*[_unwrap(a) for a in args])

    def set_materialize_grads(self, value):
        self._tctx.set_materialize_grads(value)

    def __setattr__(self, k, v):
        object.__setattr__(self, k, v)


def _make_function(layer_cls):
    class _Fn(torch.autograd.Function):
        @staticmethod
        def forward(tctx, kwargs, mask, *args):
            ctx = PyLayerContext(tctx)
            tctx.pctx = ctx
            tctx.tensor_mask = mask
            wargs = [_wrap(a) if isinstance(a, torch.Tensor) else a for a in args]
            out = layer_cls.forward(ctx, *wargs, **kwargs)
            if isinstance(out, (tuple, list)):
                return tuple(_unwrap(o) for o in out)
            return _unwrap(out)

        @staticmethod
        def backward(tctx, *gouts):
            ctx = tctx.pctx
            g = layer_cls.backward(ctx, *[_wrap(x) if x is not None else None for x in gouts])
            if not isinstance(g, (tuple, list)):
                g = (g,)
            it = iter(None if x is None else _unwrap(x) for x in g)
            # paddle's backward returns one grad per *tensor* input
            full = [next(it, None) if is_t else None for is_t in tctx.tensor_mask]
            return (None, None, *full)

    _Fn.__name__ = layer_cls.__name__ + "Function"
    return _Fn


class _PyLayerMeta(type):
    def __init__(cls, name, bases, attrs):
        super().__init__(name, bases, attrs)
        cls._fn = None


class PyLayer(metaclass=_PyLayerMeta):
    """Custom op with user forward/backward operating on paddle Tensors."""

    @classmethod
    def apply(cls, *args, **kwargs):
        fn = cls.__dict__.get("_fn")
        if fn is None:
            fn = cls._fn = _make_function(cls)
        mask = tuple(isinstance(a, Tensor) for a in args)
        targs = [a._t if isinstance(a, Tensor) else a for a in args]
        out = fn.apply(kwargs, mask, *targs)
        if isinstance(out, tuple):
            return tuple(_wrap(o) for o in out)
        return _wrap(out)

    @staticmethod
    def forward(ctx, *args, **kwargs):
        raise NotImplementedError

    @staticmethod
    def backward(ctx, *args):
        raise NotImplementedError


EagerPyLayer = PyLayer
EagerPyLayerContext = PyLayerContext

from . import functional  # noqa: E402
from .functional import jacobian, hessian, vjp, jvp  # noqa: E402,F401
