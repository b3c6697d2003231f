"""Functional autodiff (reference: python/paddle/incubate/autograd/functional.py)."""
from __future__ import annotations

import torch

from ..framework.core import Tensor, _wrap, _unwrap

__all__ = ["jacobian", "hessian", "vjp", "jvp", "Jacobian", "Hessian"]


def _lift(func):
    def f(*ts):
        out = func(*[_wrap(t) for t in ts])
        if isinstance(out, (tuple, list)):
            return tuple(_unwrap(o) for o in out)
        return _unwrap(out)
    return f


def _as_tuple(x):
    single = isinstance(x, Tensor)
    return single, ((x,) if single else tuple(x))


def _wrap_nested(r):
    if isinstance(r, torch.Tensor):
        return _wrap(r)
    return type(r)(_wrap_nested(v) for v in r)


def vjp(func, xs, v=None):
    single, xs_ = _as_tuple(xs)
    out, g = torch.autograd.functional.vjp(_lift(func), tuple(x._t for x in xs_),
                                           None if v is None else (_unwrap(v) if isinstance(v, Tensor) else tuple(_unwrap(a) for a in v)))
    g = _wrap_nested(g)
    return _wrap_nested(out), (g[0] if single else g)


def jvp(func, xs, v=None):
    single, xs_ = _as_tuple(xs)
    vv = None if v is None else (tuple(_unwrap(a) for a in ((v,) if isinstance(v, Tensor) else v)))
    out, g = torch.autograd.functional.jvp(_lift(func), tuple(x._t for x in xs_), vv)
    return _wrap_nested(out), _wrap_nested(g)


def jacobian(func, xs, create_graph=False, allow_unused=False):
    single, xs_ = _as_tuple(xs)
    j = torch.autograd.functional.jacobian(_lift(func), tuple(x._t for x in xs_), create_graph=create_graph)
    j = _wrap_nested(j)
    if single and isinstance(j, tuple) and len(j) == 1:
        return j[0]
    return j


def hessian(func, xs, create_graph=False, allow_unused=False):
    single, xs_ = _as_tuple(xs)
    h = torch.autograd.functional.hessian(_lift(func), tuple(x._t for x in xs_), create_graph=create_graph)
    h = _wrap_nested(h)
    if single:
        while isinstance(h, tuple) and len(h) == 1:
            h = h[0]
    return h


class Jacobian:
    def __init__(self, func, xs, is_batched=False):
        self._j = jacobian(func, xs)

    def __getitem__(self, idx):
        return self._j[idx]

    @property
    def shape(self):
        return self._j.shape


class Hessian(Jacobian):
    def __init__(self, func, xs, is_batched=False):
        self._j = hessian(func, xs)
