"""nn.utils (reference: python/paddle/nn/utils/*)."""
from __future__ import annotations

import torch

from ..framework.core import Tensor, Parameter, _wrap
from .clip import clip_grad_norm_, clip_grad_value_  # noqa: F401

__all__ = ["weight_norm", "remove_weight_norm", "spectral_norm", "parameters_to_vector", "vector_to_parameters",
           "clip_grad_norm_", "clip_grad_value_"]


def _norm_except(w, dim):
    if dim is None or dim == -1:
        return w.norm()
    dims = [d for d in range(w.dim()) if d != dim]
    return w.norm(dim=dims, keepdim=True)


class _WeightNormHook:
    def __init__(self, name, dim):
        self.name, self.dim = name, dim

    def compute(self, layer):
        g = getattr(layer, self.name + "_g")._t
        v = getattr(layer, self.name + "_v")._t
        return _wrap(v * (g / _norm_except(v, self.dim)))

    def __call__(self, layer, inputs):
        object.__setattr__(layer, self.name, self.compute(layer))


def weight_norm(layer, name="weight", dim=0):
    w = getattr(layer, name)
    del layer._parameters[name]
    g = Parameter(data=_norm_except(w._t, dim).detach().clone())
    v = Parameter(data=w._t.detach().clone())
    layer.add_parameter(name + "_g", g)
    layer.add_parameter(name + "_v", v)
    hook = _WeightNormHook(name, dim)
    object.__setattr__(layer, name, hook.compute(layer))
    h = layer.register_forward_pre_hook(hook)
    layer._weight_norm_hook = (hook, h)
    return layer


def remove_weight_norm(layer, name="weight"):
    hook, h = layer._weight_norm_hook
    w = hook.compute(layer)
    h.remove()
    del layer._parameters[name + "_g"]
    del layer._parameters[name + "_v"]
    layer.__dict__.pop(name, None)
    layer.add_parameter(name, Parameter(data=w._t.detach().clone()))
    return layer


def spectral_norm(layer, name="weight", n_power_iterations=1, eps=1e-12, dim=None):
    from .layer.conv_norm_pool import SpectralNorm
    w = getattr(layer, name)
    if dim is None:
        dim = 1 if type(layer).__name__.endswith("Transpose") else 0
    sn = SpectralNorm(w.shape, dim, n_power_iterations, eps)
    del layer._parameters[name]
    layer.add_parameter(name + "_orig", w)
    layer.add_sublayer(name + "_sn", sn)

    def hook(l, inputs):
        object.__setattr__(l, name, sn(getattr(l, name + "_orig")))
    hook(layer, None)
    layer.register_forward_pre_hook(hook)
    return layer


def parameters_to_vector(parameters, name=None):
    return _wrap(torch.cat([p._t.reshape(-1) for p in parameters]))


def vector_to_parameters(vec, parameters, name=None):
    off = 0
    v = vec._t
    with torch.no_grad():
        for p in parameters:
            n = p._t.numel()
            p._t.copy_(v[off:off + n].reshape(p._t.shape))
            off += n
