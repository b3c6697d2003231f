"""``fluid.layers`` distributions (reference: python/paddle/fluid/layers/distributions.py):
Uniform, Normal and Categorical are the 2.x classes; MultivariateNormalDiag (diagonal
covariance given as a [k, k] scale matrix) is defined here."""
from __future__ import annotations

import math

import torch

from ...distribution import Uniform, Normal, Categorical  # noqa: F401
from ._common import T, W

__all__ = ["Uniform", "Normal", "Categorical", "MultivariateNormalDiag"]


class MultivariateNormalDiag:
    def __init__(self, loc, scale):
        self.loc = T(loc).float()
        s = T(scale).float()
        self.var = torch.diagonal(s, dim1=-2, dim2=-1) if s.dim() >= 2 else s

    def _det(self):
        return self.var.prod(-1)

    def entropy(self):
        k = self.loc.shape[-1]
        return W(0.5 * (k * (1.0 + math.log(2 * math.pi)) + torch.log(self._det())))

    def kl_divergence(self, other):
        tr = (self.var / other.var).sum(-1)
        d = other.loc - self.loc
        maha = (d * d / other.var).sum(-1)
        k = self.loc.shape[-1]
        return W(0.5 * (tr + maha - k + torch.log(other._det() / self._det())))

    def sample(self, shape, seed=0):
        g = torch.Generator(device=self.loc.device)
        if seed:
            g.manual_seed(int(seed))
        eps = torch.randn(list(shape) + list(self.loc.shape), generator=g, device=self.loc.device)
        return W(self.loc + eps * self.var.sqrt())

    def log_prob(self, value):
        v = T(value).float()
        d = v - self.loc
        k = self.loc.shape[-1]
        return W(-0.5 * ((d * d / self.var).sum(-1) + k * math.log(2 * math.pi) + torch.log(self._det())))
