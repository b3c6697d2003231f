"""Random ops + global seeding (reference: python/paddle/tensor/random.py,
python/paddle/framework/random.py). One torch generator per HIP device; the
tensor-parallel RNG tracker (parallel/mp_layers.py) swaps generator states."""
from __future__ import annotations

import numpy as np
import torch

from ..framework import core as _core
from ..framework.core import Tensor, convert_dtype, default_device
from ..framework.dispatch import register_ops
from ._helpers import _u, _w, _int_list, _dtype_or_default

__all__ = ["bernoulli", "poisson", "multinomial", "standard_normal", "normal", "uniform",
           "randn", "rand", "randint", "randint_like", "randperm", "uniform_", "exponential_",
           "normal_", "seed", "get_cuda_rng_state", "set_cuda_rng_state", "get_rng_state",
           "set_rng_state"]


def seed(s):
    s = int(s)
    np.random.seed(s % (2 ** 32))
    torch.manual_seed(s)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(s)
    import random as _r
    _r.seed(s)
    return torch.default_generator


def get_cuda_rng_state():
    return [torch.cuda.get_rng_state(i) for i in range(torch.cuda.device_count())] if torch.cuda.is_available() else []


def set_cuda_rng_state(state_list):
    for i, s in enumerate(state_list):
        torch.cuda.set_rng_state(s, i)


def get_rng_state(device=None):
    return [torch.get_rng_state()] + get_cuda_rng_state()


def set_rng_state(state_list, device=None):
    torch.set_rng_state(state_list[0])
    set_cuda_rng_state(state_list[1:])


def _shape(shape):
    return _int_list(shape)


def bernoulli(x, name=None):
    return _w(torch.bernoulli(_u(x)))


def poisson(x, name=None):
    return _w(torch.poisson(_u(x)))


def multinomial(x, num_samples=1, replacement=False, name=None):
    return _w(torch.multinomial(_u(x), num_samples, replacement))


def standard_normal(shape, dtype=None, name=None):
    return _w(torch.randn(_shape(shape), dtype=_dtype_or_default(dtype), device=default_device()))


def randn(shape, dtype=None, name=None):
    return standard_normal(shape, dtype)


def normal(mean=0.0, std=1.0, shape=None, name=None):
    if isinstance(mean, Tensor) or isinstance(std, Tensor):
        m, s = _u(mean), _u(std)
        if not isinstance(m, torch.Tensor):
            m = torch.full_like(s, m)
        if not isinstance(s, torch.Tensor):
            s = torch.full_like(m, s)
        return _w(torch.normal(m, s))
    return _w(torch.normal(mean, std, _shape(shape), dtype=_core._default_dtype, device=default_device()))


def normal_(x, mean=0.0, std=1.0, name=None):
    with torch.no_grad():
        x._t.normal_(mean, std)
    return x


def uniform(shape, dtype=None, min=-1.0, max=1.0, seed=0, name=None):
    g = None
    dev = default_device()
    if seed:
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
    t = torch.empty(_shape(shape), dtype=_dtype_or_default(dtype), device=dev)
    t.uniform_(min, max, generator=g)
    return _w(t)


def uniform_(x, min=-1.0, max=1.0, seed=0, name=None):
    with torch.no_grad():
        x._t.uniform_(min, max)
    return x


def exponential_(x, lam=1.0, name=None):
    with torch.no_grad():
        x._t.exponential_(lam)
    return x


def rand(shape, dtype=None, name=None):
    return _w(torch.rand(_shape(shape), dtype=_dtype_or_default(dtype), device=default_device()))


def randint(low=0, high=None, shape=[1], dtype=None, name=None):
    if high is None:
        low, high = 0, low
    dt = convert_dtype(dtype) or torch.int64
    return _w(torch.randint(low, high, _shape(shape), dtype=dt, device=default_device()))


def randint_like(x, low=0, high=None, dtype=None, name=None):
    if high is None:
        low, high = 0, low
    t = _u(x)
    dt = convert_dtype(dtype) or t.dtype
    return _w(torch.randint(low, high, t.shape, device=t.device).to(dt))


def randperm(n, dtype="int64", name=None):
    return _w(torch.randperm(n, dtype=convert_dtype(dtype), device=default_device()))


register_ops(globals(), ["bernoulli", "poisson", "multinomial", "normal", "normal_", "uniform_",
                         "exponential_", "randint_like"])


def gaussian(shape, mean=0.0, std=1.0, dtype=None, name=None):
    """(reference: tensor/random.py gaussian) samples of N(mean, std^2) with ``shape``"""
    from .. import normal
    out = normal(mean, std, shape)
    return out.astype(dtype) if dtype is not None else out
