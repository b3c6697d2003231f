"""incubate.autograd (reference: python/paddle/incubate/autograd/{functional,primapi,primx}.py).

``enable_prim``/``disable_prim`` toggle the reference's primitive-operator autodiff for
static programs; here autodiff is always torch's tape (which already decomposes into
primitive backward kernels), so the switch is recorded and ``forward_grad``/``grad``
are computed with forward-mode (jvp) / reverse-mode autodiff directly."""
from __future__ import annotations

import torch

from ...framework.core import Tensor, _wrap
from ...autograd.functional import vjp, jvp, Jacobian, Hessian  # noqa: F401

__all__ = ["vjp", "jvp", "Jacobian", "Hessian", "enable_prim", "disable_prim", "forward_grad", "grad",
           "prim_enabled"]

_prim = False


def enable_prim():
    global _prim
    _prim = True


def disable_prim():
    global _prim
    _prim = False


def prim_enabled():
    return _prim


def _list(x):
    return (list(x), False) if isinstance(x, (list, tuple)) else ([x], True)


def grad(outputs, inputs, grad_outputs=None):
    outs, _ = _list(outputs)
    ins, single = _list(inputs)
    if grad_outputs is not None:
        gos = [g._t if isinstance(g, Tensor) else g for g in _list(grad_outputs)[0]]
    else:
        gos = [torch.ones_like(o._t) for o in outs]
    gs = torch.autograd.grad([o._t for o in outs], [i._t for i in ins], gos, retain_graph=True, allow_unused=True,
                             create_graph=True)
    res = [_wrap(g) if g is not None else None for g in gs]
    return res[0] if single else res


def forward_grad(outputs, inputs, grad_inputs=None):
    """Forward-mode derivative d(outputs)/d(inputs) · grad_inputs via the double-vjp trick
    (works on any recorded graph without re-running the function)."""
    outs, single_out = _list(outputs)
    ins, _ = _list(inputs)
    tangents = [torch.ones_like(i._t) if grad_inputs is None else g._t
                for i, g in zip(ins, _list(grad_inputs)[0] if grad_inputs is not None else ins)]
    us = [torch.zeros_like(o._t, requires_grad=True) for o in outs]
    gs = torch.autograd.grad([o._t for o in outs], [i._t for i in ins], us, create_graph=True, allow_unused=True)
    pairs = [(g, t) for g, t in zip(gs, tangents) if g is not None]
    res = torch.autograd.grad([g for g, _ in pairs], us, [t for _, t in pairs], create_graph=True, allow_unused=True)
    res = [_wrap(r) if r is not None else None for r in res]
    return res[0] if single_out else res
