"""``paddle.distribution`` (reference: python/paddle/distribution/*.py).

Distributions hold torch tensors (so samples/log-probs are differentiable through the
reparameterised paths and run on the MI355X when the parameters live there) and return
framework Tensors. Semantics follow the reference, including its quirks: ``Categorical``
treats ``logits`` as unnormalised probabilities in ``probs``/``sample`` but as logits in
``entropy``/``kl_divergence`` (reference categorical.py:118, 257).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..framework.core import Tensor, _wrap, default_device, convert_dtype
from . import transform  # noqa: F401
from .transform import *  # noqa: F401,F403

__all__ = ["Beta", "Categorical", "Dirichlet", "Distribution", "ExponentialFamily", "Multinomial", "Normal",
           "Uniform", "kl_divergence", "register_kl", "Independent", "TransformedDistribution"] + transform.__all__


def _t(x, dtype=torch.float32):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    a = np.asarray(x)
    if a.dtype == np.float64 and dtype == torch.float32:
        a = a.astype(np.float32)
    return torch.as_tensor(a, device=default_device()).to(dtype if not np.issubdtype(a.dtype, np.floating)
                                                        or a.dtype == np.float32 else torch.from_numpy(a[:0]).dtype)


def _shape(s):
    return tuple(int(v) for v in (s if isinstance(s, (list, tuple)) else [s]))


class Distribution:
    def __init__(self, batch_shape=(), event_shape=()):
        self._batch_shape = tuple(batch_shape)
        self._event_shape = tuple(event_shape)

    @property
    def batch_shape(self):
        return self._batch_shape

    @property
    def event_shape(self):
        return self._event_shape

    @property
    def mean(self):
        raise NotImplementedError

    @property
    def variance(self):
        raise NotImplementedError

    def sample(self, shape=()):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape=()):
        raise NotImplementedError

    def entropy(self):
        raise NotImplementedError

    def kl_divergence(self, other):
        return kl_divergence(self, other)

    def prob(self, value):
        return _wrap(torch.exp(self.log_prob(value)._t))

    def probs(self, value):
        return self.prob(value)

    def log_prob(self, value):
        raise NotImplementedError

    def _extend_shape(self, sample_shape):
        return _shape(sample_shape) + self._batch_shape + self._event_shape

    def _validate_args(self, *args):
        return True

    def _to_tensor(self, *args):
        return tuple(_t(a) for a in args)


class ExponentialFamily(Distribution):
    """Entropy via the Bregman divergence of the log-normaliser (reference exponential_family.py)."""

    @property
    def _natural_parameters(self):
        raise NotImplementedError

    def _log_normalizer(self, *natural):
        raise NotImplementedError

    @property
    def _mean_carrier_measure(self):
        raise NotImplementedError

    def entropy(self):
        nat = [p.detach().requires_grad_() for p in self._natural_parameters]
        with torch.enable_grad():
            lg = self._log_normalizer(*nat)
            grads = torch.autograd.grad(lg.sum(), nat, create_graph=True)
        ent = -self._mean_carrier_measure + lg
        for p, g in zip(nat, grads):
            term = p * g
            if term.dim() > lg.dim():
                term = term.sum(tuple(range(lg.dim() - term.dim(), 0)))
            ent = ent - term
        return _wrap(ent)


class Normal(Distribution):
    def __init__(self, loc, scale, name=None):
        self.loc, self.scale = torch.broadcast_tensors(_t(loc), _t(scale))
        self.name = name or "Normal"
        super().__init__(self.loc.shape)

    mean = property(lambda s: _wrap(s.loc))
    variance = property(lambda s: _wrap(s.scale ** 2))

    def rsample(self, shape=(), seed=0):
        s = self._extend_shape(shape)
        eps = torch.randn(s, dtype=self.loc.dtype, device=self.loc.device)
        return _wrap(self.loc + eps * self.scale)

    def sample(self, shape=(), seed=0):
        with torch.no_grad():
            return self.rsample(shape)

    def entropy(self):
        return _wrap(0.5 + 0.5 * math.log(2 * math.pi) + torch.log(self.scale))

    def log_prob(self, value):
        v = _t(value).to(self.loc.dtype)
        var = self.scale ** 2
        return _wrap(-((v - self.loc) ** 2) / (2 * var) - torch.log(self.scale) - math.log(math.sqrt(2 * math.pi)))

    def probs(self, value):
        return _wrap(torch.exp(self.log_prob(value)._t))


class Uniform(Distribution):
    def __init__(self, low, high, name=None):
        self.low, self.high = torch.broadcast_tensors(_t(low), _t(high))
        self.name = name or "Uniform"
        super().__init__(self.low.shape)

    mean = property(lambda s: _wrap((s.low + s.high) / 2))
    variance = property(lambda s: _wrap((s.high - s.low) ** 2 / 12))

    def rsample(self, shape=(), seed=0):
        u = torch.rand(self._extend_shape(shape), dtype=self.low.dtype, device=self.low.device)
        return _wrap(self.low + u * (self.high - self.low))

    def sample(self, shape=(), seed=0):
        with torch.no_grad():
            return self.rsample(shape)

    def log_prob(self, value):
        v = _t(value).to(self.low.dtype)
        inside = ((v > self.low) & (v < self.high)).to(v.dtype)
        return _wrap(torch.log(inside) - torch.log(self.high - self.low))

    def probs(self, value):
        v = _t(value).to(self.low.dtype)
        inside = ((v > self.low) & (v < self.high)).to(v.dtype)
        return _wrap(inside / (self.high - self.low))

    def entropy(self):
        return _wrap(torch.log(self.high - self.low))


class Categorical(Distribution):
    def __init__(self, logits, name=None):
        self.logits = _t(logits)
        if not self.logits.is_floating_point():
            self.logits = self.logits.float()
        self._prob = self.logits / self.logits.sum(-1, keepdim=True)
        self.name = name or "Categorical"
        super().__init__(self.logits.shape[:-1])

    def sample(self, shape=()):
        shape = _shape(shape)
        n = int(np.prod(shape)) if shape else 1
        flat = self._prob.reshape(-1, self._prob.shape[-1])
        idx = torch.multinomial(flat, n, replacement=True)  # [B, n]
        out = idx.t().reshape(shape + tuple(self._prob.shape[:-1]))
        return _wrap(out)

    def _softmax(self):
        lg = self.logits - self.logits.max(-1, keepdim=True).values
        e = torch.exp(lg)
        z = e.sum(-1, keepdim=True)
        return lg, z, e / z

    def entropy(self):
        lg, z, p = self._softmax()
        return _wrap(-(p * (lg - torch.log(z))).sum(-1, keepdim=True))

    def kl_divergence(self, other):
        lg, z, p = self._softmax()
        olg, oz, _ = other._softmax()
        return _wrap((p * (lg - torch.log(z) - olg + torch.log(oz))).sum(-1, keepdim=True))

    def probs(self, value):
        v = _t(value, torch.int64).long()
        if self._prob.dim() == 1:
            return _wrap(self._prob[v])
        if v.dim() == self._prob.dim() - 1 or v.shape[:-1] != self._prob.shape[:-1]:
            # one index set applied to every distribution in the batch
            return _wrap(torch.gather(self._prob, -1, v.reshape(1, -1).expand(self._prob.shape[0], -1)
                                      if self._prob.dim() == 2 else v))
        return _wrap(torch.gather(self._prob, -1, v))

    def log_prob(self, value):
        return _wrap(torch.log(self.probs(value)._t))


class Beta(ExponentialFamily):
    def __init__(self, alpha, beta):
        self.alpha, self.beta = torch.broadcast_tensors(_t(alpha), _t(beta))
        self._dirichlet = torch.stack([self.alpha, self.beta], -1)
        super().__init__(self.alpha.shape)

    mean = property(lambda s: _wrap(s.alpha / (s.alpha + s.beta)))
    variance = property(lambda s: _wrap(s.alpha * s.beta / ((s.alpha + s.beta) ** 2 * (s.alpha + s.beta + 1))))

    def prob(self, value):
        return _wrap(torch.exp(self.log_prob(value)._t))

    def log_prob(self, value):
        v = _t(value).to(self.alpha.dtype)
        a, b = self.alpha, self.beta
        return _wrap((a - 1) * torch.log(v) + (b - 1) * torch.log1p(-v) - (torch.lgamma(a) + torch.lgamma(b)
                                                                           - torch.lgamma(a + b)))

    def sample(self, shape=()):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape=()):
        d = torch.distributions.Beta(self.alpha, self.beta)
        return _wrap(d.rsample(_shape(shape) if shape != () else ()))

    def entropy(self):
        return _wrap(torch.distributions.Beta(self.alpha, self.beta).entropy())

    @property
    def _natural_parameters(self):
        return (self.alpha, self.beta)

    def _log_normalizer(self, x, y):
        return torch.lgamma(x) + torch.lgamma(y) - torch.lgamma(x + y)

    _mean_carrier_measure = 0


class Dirichlet(ExponentialFamily):
    def __init__(self, concentration):
        self.concentration = _t(concentration)
        if self.concentration.dim() < 1:
            raise ValueError("`concentration` parameter must be at least one dimensional")
        super().__init__(self.concentration.shape[:-1], self.concentration.shape[-1:])

    mean = property(lambda s: _wrap(s.concentration / s.concentration.sum(-1, keepdim=True)))

    @property
    def variance(self):
        c0 = self.concentration.sum(-1, keepdim=True)
        return _wrap(self.concentration * (c0 - self.concentration) / (c0 ** 2 * (c0 + 1)))

    def sample(self, shape=()):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape=()):
        return _wrap(torch.distributions.Dirichlet(self.concentration).rsample(_shape(shape) if shape != () else ()))

    def prob(self, value):
        return _wrap(torch.exp(self.log_prob(value)._t))

    def log_prob(self, value):
        v = _t(value).to(self.concentration.dtype)
        c = self.concentration
        return _wrap(((c - 1) * torch.log(v)).sum(-1) + torch.lgamma(c.sum(-1)) - torch.lgamma(c).sum(-1))

    def entropy(self):
        return _wrap(torch.distributions.Dirichlet(self.concentration).entropy())

    @property
    def _natural_parameters(self):
        return (self.concentration,)

    def _log_normalizer(self, x):
        return torch.lgamma(x).sum(-1) - torch.lgamma(x.sum(-1))

    _mean_carrier_measure = 0


class Multinomial(Distribution):
    def __init__(self, total_count, probs):
        if not isinstance(total_count, int) or total_count < 1:
            raise ValueError("input parameter total_count must be int type and greater than 0")
        self.total_count = total_count
        p = _t(probs)
        self.probs_t = p / p.sum(-1, keepdim=True)
        self._categorical = Categorical(torch.log(self.probs_t))
        super().__init__(self.probs_t.shape[:-1], self.probs_t.shape[-1:])

    mean = property(lambda s: _wrap(s.probs_t * s.total_count))
    variance = property(lambda s: _wrap(s.total_count * s.probs_t * (1 - s.probs_t)))

    def prob(self, value):
        return _wrap(torch.exp(self.log_prob(value)._t))

    def log_prob(self, value):
        v = _t(value).to(self.probs_t.dtype)
        logp = torch.log(self.probs_t.clamp_min(torch.finfo(self.probs_t.dtype).tiny))
        return _wrap(torch.lgamma(v.sum(-1) + 1) - torch.lgamma(v + 1).sum(-1) + (v * logp).sum(-1))

    def sample(self, shape=()):
        shape = _shape(shape) if shape != () else ()
        flat = self.probs_t.reshape(-1, self.probs_t.shape[-1])
        n = int(np.prod(shape)) if shape else 1
        draws = torch.multinomial(flat, self.total_count * n, replacement=True).reshape(flat.shape[0], n,
                                                                                        self.total_count)
        counts = torch.zeros(flat.shape[0], n, flat.shape[1], dtype=self.probs_t.dtype, device=flat.device)
        counts.scatter_add_(-1, draws, torch.ones_like(draws, dtype=counts.dtype))
        counts = counts.permute(1, 0, 2).reshape(shape + tuple(self.probs_t.shape))
        return _wrap(counts)

    def entropy(self):
        return _wrap(torch.distributions.Multinomial(self.total_count, probs=self.probs_t).entropy())


class Independent(Distribution):
    def __init__(self, base, reinterpreted_batch_rank):
        if not 0 < reinterpreted_batch_rank <= len(base.batch_shape):
            raise ValueError("Expected 0 < reinterpreted_batch_rank <= len(base.batch_shape)")
        self._base = base
        self._rank = reinterpreted_batch_rank
        k = len(base.batch_shape) - reinterpreted_batch_rank
        super().__init__(base.batch_shape[:k], base.batch_shape[k:] + base.event_shape)

    mean = property(lambda s: s._base.mean)
    variance = property(lambda s: s._base.variance)

    def sample(self, shape=()):
        return self._base.sample(shape)

    def rsample(self, shape=()):
        return self._base.rsample(shape)

    def _sum_rightmost(self, t):
        return t.sum(tuple(range(-self._rank, 0))) if self._rank > 0 else t

    def log_prob(self, value):
        return _wrap(self._sum_rightmost(self._base.log_prob(value)._t))

    def prob(self, value):
        return _wrap(torch.exp(self.log_prob(value)._t))

    def entropy(self):
        return _wrap(self._sum_rightmost(self._base.entropy()._t))


class TransformedDistribution(Distribution):
    def __init__(self, base, transforms):
        if not isinstance(base, Distribution):
            raise TypeError("base must be a Distribution")
        self._base = base
        self._transforms = list(transforms)
        chain = transform.ChainTransform(self._transforms)
        shape = base.batch_shape + base.event_shape
        out_shape = chain.forward_shape(shape)
        ev = max(len(base.event_shape), chain._codomain_event_rank())
        super().__init__(tuple(out_shape[:len(out_shape) - ev]), tuple(out_shape[len(out_shape) - ev:]))

    def sample(self, shape=()):
        x = self._base.sample(shape)
        for t in self._transforms:
            x = t.forward(x)
        return x

    def rsample(self, shape=()):
        x = self._base.rsample(shape)
        for t in self._transforms:
            x = t.forward(x)
        return x

    def log_prob(self, value):
        y = value if isinstance(value, Tensor) else _wrap(_t(value))
        lp = 0.0
        ev = len(self.event_shape)
        for t in reversed(self._transforms):
            x = t.inverse(y)
            ldj = t.forward_log_det_jacobian(x)._t
            extra = ev - t._codomain.event_rank
            if extra > 0:
                ldj = ldj.sum(tuple(range(-extra, 0)))
            lp = lp - ldj
            ev += t._domain.event_rank - t._codomain.event_rank
            y = x
        base_lp = self._base.log_prob(y)._t
        extra = ev - len(self._base.event_shape)
        if extra > 0:
            base_lp = base_lp.sum(tuple(range(-extra, 0)))
        return _wrap(base_lp + lp)

    def prob(self, value):
        return _wrap(torch.exp(self.log_prob(value)._t))


# --------------------------------------------------------------------------- KL registry
_KL = {}


def register_kl(cls_p, cls_q):
    if not (issubclass(cls_p, Distribution) and issubclass(cls_q, Distribution)):
        raise TypeError("cls_p and cls_q must be subclass of Distribution")

    def deco(f):
        _KL[(cls_p, cls_q)] = f
        return f
    return deco


def _dispatch(tp, tq):
    matches = [(p, q) for (p, q) in _KL if issubclass(tp, p) and issubclass(tq, q)]
    if not matches:
        return None
    # most specific match (shortest MRO distance)
    return _KL[min(matches, key=lambda pq: (tp.__mro__.index(pq[0]), tq.__mro__.index(pq[1])))]


def kl_divergence(p, q):
    f = _dispatch(type(p), type(q))
    if f is None:
        raise NotImplementedError(f"KL divergence of {type(p).__name__} and {type(q).__name__} is not registered")
    return f(p, q)


@register_kl(Normal, Normal)
def _kl_normal(p, q):
    var_ratio = (p.scale / q.scale) ** 2
    t1 = ((p.loc - q.loc) / q.scale) ** 2
    return _wrap(0.5 * (var_ratio + t1 - 1 - torch.log(var_ratio)))


@register_kl(Uniform, Uniform)
def _kl_uniform(p, q):
    res = torch.log((q.high - q.low) / (p.high - p.low))
    bad = (q.low > p.low) | (q.high < p.high)
    return _wrap(torch.where(bad, torch.full_like(res, float("inf")), res))


@register_kl(Categorical, Categorical)
def _kl_categorical(p, q):
    return p.kl_divergence(q)


@register_kl(Beta, Beta)
def _kl_beta(p, q):
    return _wrap(torch.distributions.kl_divergence(torch.distributions.Beta(p.alpha, p.beta),
                                                   torch.distributions.Beta(q.alpha, q.beta)))


@register_kl(Dirichlet, Dirichlet)
def _kl_dirichlet(p, q):
    return _wrap(torch.distributions.kl_divergence(torch.distributions.Dirichlet(p.concentration),
                                                   torch.distributions.Dirichlet(q.concentration)))


@register_kl(ExponentialFamily, ExponentialFamily)
def _kl_expfamily(p, q):
    """Bregman divergence of the log-normaliser (reference kl.py:_kl_expfamily_expfamily)."""
    if type(p) is not type(q):
        raise NotImplementedError
    pn = [t.detach().requires_grad_() for t in p._natural_parameters]
    qn = list(q._natural_parameters)
    with torch.enable_grad():
        lp = p._log_normalizer(*pn)
        grads = torch.autograd.grad(lp.sum(), pn)
    kl = q._log_normalizer(*qn) - lp.detach()
    for a, b, g in zip(pn, qn, grads):
        term = (b - a.detach()) * g
        kl = kl + (term.sum(-1) if term.dim() > kl.dim() else term)
    return _wrap(kl)
