"""Quasi-Newton minimisers (reference: python/paddle/incubate/optimizer/functional/{bfgs,lbfgs}.py).

Both return ``(is_converge, num_func_calls, position, objective_value, objective_gradient
[, inverse_hessian_estimate])`` like the reference; line search is strong-Wolfe (zoom)."""
from __future__ import annotations

import torch

from ...framework.core import Tensor, _wrap

__all__ = ["minimize_bfgs", "minimize_lbfgs"]


def _fg(fn, x):
    x = x.detach().requires_grad_(True)
    with torch.enable_grad():
        out = fn(_wrap(x))
        f = out._t if isinstance(out, Tensor) else out
        g, = torch.autograd.grad(f, x)
    return f.detach(), g.detach()


def _wolfe(fn, x, f0, g0, d, a_init=1.0, c1=1e-4, c2=0.9, max_iters=50):
    """Strong-Wolfe line search with bisection zoom. Returns (alpha, f, g, ncalls)."""
    dg0 = (g0 * d).sum()
    lo, hi = 0.0, None
    a = a_init
    f_lo = f0
    calls = 0
    for _ in range(max_iters):
        f, g = _fg(fn, x + a * d)
        calls += 1
        dg = (g * d).sum()
        if f > f0 + c1 * a * dg0 or (hi is None and f >= f_lo and lo > 0):
            hi = a
        elif abs(dg) <= -c2 * dg0:
            return a, f, g, calls
        elif dg * ((hi if hi is not None else 2 * a) - lo) >= 0:
            hi = lo
            lo, f_lo = a, f
        else:
            lo, f_lo = a, f
        a = (lo + hi) / 2 if hi is not None else 2 * a
    return a, f, g, calls


def minimize_bfgs(objective_func, initial_position, max_iters=50, tolerance_grad=1e-7, tolerance_change=1e-9,
                  initial_inverse_hessian_estimate=None, line_search_fn="strong_wolfe", max_line_search_iters=50,
                  initial_step_length=1.0, dtype="float32", name=None):
    x = (initial_position._t if isinstance(initial_position, Tensor) else torch.as_tensor(initial_position)).detach()
    dt = torch.float64 if dtype == "float64" else torch.float32
    x = x.to(dt)
    n = x.numel()
    H = (initial_inverse_hessian_estimate._t.to(dt) if initial_inverse_hessian_estimate is not None
         else torch.eye(n, dtype=dt, device=x.device))
    f, g = _fg(objective_func, x)
    calls = 1
    converged = bool(g.abs().max() <= tolerance_grad)
    for _ in range(max_iters):
        if converged:
            break
        d = -(H @ g.reshape(-1)).reshape(x.shape)
        a, f_new, g_new, c = _wolfe(objective_func, x, f, g, d, initial_step_length, max_iters=max_line_search_iters)
        calls += c
        s = (a * d).reshape(-1)
        y = (g_new - g).reshape(-1)
        x = x + a * d
        ys = y @ s
        if ys > 1e-10:
            rho = 1.0 / ys
            I = torch.eye(n, dtype=dt, device=x.device)
            V = I - rho * torch.outer(s, y)
            H = V @ H @ V.t() + rho * torch.outer(s, s)
        change = (f - f_new).abs()
        f, g = f_new, g_new
        if g.abs().max() <= tolerance_grad or change <= tolerance_change or s.abs().max() <= tolerance_change:
            converged = True
    return (_wrap(torch.tensor(converged)), _wrap(torch.tensor(calls)), _wrap(x), _wrap(f), _wrap(g), _wrap(H))


def minimize_lbfgs(objective_func, initial_position, history_size=100, max_iters=50, tolerance_grad=1e-8,
                   tolerance_change=1e-8, initial_inverse_hessian_estimate=None, line_search_fn="strong_wolfe",
                   max_line_search_iters=50, initial_step_length=1.0, dtype="float32", name=None):
    x = (initial_position._t if isinstance(initial_position, Tensor) else torch.as_tensor(initial_position)).detach()
    dt = torch.float64 if dtype == "float64" else torch.float32
    x = x.to(dt)
    f, g = _fg(objective_func, x)
    calls = 1
    S, Y = [], []
    converged = bool(g.abs().max() <= tolerance_grad)
    for _ in range(max_iters):
        if converged:
            break
        q = g.reshape(-1).clone()
        alphas = []
        for s, y in reversed(list(zip(S, Y))):
            rho = 1.0 / (y @ s)
            a = rho * (s @ q)
            q -= a * y
            alphas.append((a, rho))
        gamma = (S[-1] @ Y[-1]) / (Y[-1] @ Y[-1]) if S else 1.0
        r = gamma * q
        for (s, y), (a, rho) in zip(zip(S, Y), reversed(alphas)):
            b = rho * (y @ r)
            r += s * (a - b)
        d = -r.reshape(x.shape)
        a, f_new, g_new, c = _wolfe(objective_func, x, f, g, d, initial_step_length, max_iters=max_line_search_iters)
        calls += c
        s = (a * d).reshape(-1)
        y = (g_new - g).reshape(-1)
        x = x + a * d
        if y @ s > 1e-10:
            S.append(s)
            Y.append(y)
            if len(S) > history_size:
                S.pop(0)
                Y.pop(0)
        change = (f - f_new).abs()
        f, g = f_new, g_new
        if g.abs().max() <= tolerance_grad or change <= tolerance_change or s.abs().max() <= tolerance_change:
            converged = True
    return (_wrap(torch.tensor(converged)), _wrap(torch.tensor(calls)), _wrap(x), _wrap(f), _wrap(g))
