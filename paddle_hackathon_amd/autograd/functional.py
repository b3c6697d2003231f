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
    """v defaults to all-ones cotangents (reference semantics), for any output shape."""
    single, xs_ = _as_tuple(xs)
    if v is None:
        with torch.no_grad():
            o = _lift(func)(*[x._t for x in xs_])
        v = tuple(torch.ones_like(t) for t in (o if isinstance(o, tuple) else (o,)))
        v = v[0] if len(v) == 1 else v
    else:
        v = _unwrap(v) if isinstance(v, Tensor) else tuple(_unwrap(a) for a in v)
    out, g = torch.autograd.functional.vjp(_lift(func), tuple(x._t for x in xs_), v)
    g = _wrap_nested(g)
    return _wrap_nested(out), (g[0] if single else g)


def jvp(func, xs, v=None):
    single, xs_ = _as_tuple(xs)
    vv = (tuple(torch.ones_like(x._t) for x in xs_) if v is None
          else tuple(_unwrap(a) for a in ((v,) if isinstance(v, Tensor) else v)))
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
    """Lazily-indexable Jacobian matrix (reference incubate/autograd/functional.py:Jacobian).

    Non-batched: shape [M, N], M = numel of all outputs, N = numel of all inputs
    (multiple inputs/outputs are flattened and concatenated). Batched (``is_batched``):
    inputs/outputs carry a leading batch dim B and the shape is [B, M, N]."""

    def __init__(self, func, xs, is_batched=False):
        self._func, self._batched = func, is_batched
        _, self._xs = _as_tuple(xs)
        self._mat = None

    def _compute(self):
        if self._mat is not None:
            return self._mat
        xs = tuple(x._t for x in self._xs)
        f = _lift(self._func)

        def flat(*ts):
            out = f(*ts)
            outs = out if isinstance(out, tuple) else (out,)
            if self._batched:
                return torch.cat([o.reshape(o.shape[0], -1) for o in outs], 1)
            return torch.cat([o.reshape(-1) for o in outs])

        j = torch.autograd.functional.jacobian(flat, xs)
        if self._batched:
            # j[i]: [B, M, B, n_i] -> take the diagonal over batch
            mats = []
            for ji in j:
                B = ji.shape[0]
                d = ji.reshape(B, ji.shape[1], B, -1)
                mats.append(torch.stack([d[b, :, b] for b in range(B)]))
            self._mat = torch.cat(mats, -1)
        else:
            self._mat = torch.cat([ji.reshape(ji.shape[0], -1) for ji in j], 1)
        return self._mat

    def __getitem__(self, idx):
        return _wrap(self._compute()[idx])

    @property
    def shape(self):
        return list(self._compute().shape)


class Hessian(Jacobian):
    """Hessian of a scalar function as a [N, N] (or batched [B, N, N]) matrix."""

    def __init__(self, func, xs, is_batched=False):
        def grad_fn(*xs_):
            ts = [x._t if isinstance(x, Tensor) else x for x in xs_]
            with torch.enable_grad():
                out = _lift(func)(*ts)
                gs = torch.autograd.grad(out.sum() if self_batched else out, ts, create_graph=True)
            return tuple(_wrap(g) for g in gs) if len(gs) > 1 else _wrap(gs[0])
        self_batched = is_batched
        super().__init__(grad_fn, xs, is_batched)
