"""Bijective transforms for ``TransformedDistribution`` (reference:
python/paddle/distribution/transform.py, variable.py). Each transform works on framework
Tensors (and numpy/torch inputs) and reports domain/codomain event ranks."""
from __future__ import annotations

import enum
import math
import operator
import functools

import torch
import torch.nn.functional as TF

from ..framework.core import Tensor, _wrap

__all__ = ["Transform", "AbsTransform", "AffineTransform", "ChainTransform", "ExpTransform", "IndependentTransform",
           "PowerTransform", "ReshapeTransform", "SigmoidTransform", "SoftmaxTransform", "StackTransform",
           "StickBreakingTransform", "TanhTransform"]


def _u(x):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    return torch.as_tensor(x, dtype=torch.float32)


class _Var:
    def __init__(self, is_discrete=False, event_rank=0):
        self.is_discrete = is_discrete
        self.event_rank = event_rank


class Type(enum.Enum):
    BIJECTION = "bijection"
    INJECTION = "injection"
    SURJECTION = "surjection"
    OTHER = "other"

    @classmethod
    def is_injective(cls, t):
        return t in (cls.BIJECTION, cls.INJECTION)


class Transform:
    _type = Type.INJECTION
    _domain = _Var()
    _codomain = _Var()

    def __call__(self, x):
        if isinstance(x, Transform):
            return ChainTransform([self, x])
        return self.forward(x)

    @classmethod
    def _is_injective(cls):
        return Type.is_injective(cls._type)

    def forward(self, x):
        return _wrap(self._forward(_u(x)))

    def inverse(self, y):
        return _wrap(self._inverse(_u(y)))

    def forward_log_det_jacobian(self, x):
        return _wrap(self._forward_log_det_jacobian(_u(x)))

    def inverse_log_det_jacobian(self, y):
        yt = _u(y)
        return _wrap(-self._forward_log_det_jacobian(self._inverse(yt)))

    def forward_shape(self, shape):
        return tuple(shape)

    def inverse_shape(self, shape):
        return tuple(shape)

    def _codomain_event_rank(self):
        return self._codomain.event_rank

    def _forward(self, x):
        raise NotImplementedError

    def _inverse(self, y):
        raise NotImplementedError

    def _forward_log_det_jacobian(self, x):
        raise NotImplementedError


class AbsTransform(Transform):
    _type = Type.SURJECTION

    def _forward(self, x):
        return x.abs()

    def inverse(self, y):
        t = _u(y)
        return _wrap(-t), _wrap(t)

    def inverse_log_det_jacobian(self, y):
        z = torch.zeros_like(_u(y))
        return _wrap(z), _wrap(z)

    def _forward_log_det_jacobian(self, x):
        return torch.zeros_like(x)


class AffineTransform(Transform):
    _type = Type.BIJECTION

    def __init__(self, loc, scale):
        self.loc, self.scale = _u(loc), _u(scale)

    def _forward(self, x):
        return self.loc + self.scale * x

    def _inverse(self, y):
        return (y - self.loc) / self.scale

    def _forward_log_det_jacobian(self, x):
        return torch.log(self.scale.abs()).expand_as(x) if self.scale.dim() <= x.dim() else torch.log(self.scale.abs())

    def forward_shape(self, shape):
        return tuple(torch.broadcast_shapes(tuple(shape), tuple(self.loc.shape), tuple(self.scale.shape)))

    inverse_shape = forward_shape


class ExpTransform(Transform):
    _type = Type.BIJECTION

    def _forward(self, x):
        return x.exp()

    def _inverse(self, y):
        return y.log()

    def _forward_log_det_jacobian(self, x):
        return x


class PowerTransform(Transform):
    _type = Type.BIJECTION

    def __init__(self, power):
        self.power = _u(power)

    def _forward(self, x):
        return x.pow(self.power)

    def _inverse(self, y):
        return y.pow(1 / self.power)

    def _forward_log_det_jacobian(self, x):
        return torch.log((self.power * x.pow(self.power - 1)).abs())

    def forward_shape(self, shape):
        return tuple(torch.broadcast_shapes(tuple(shape), tuple(self.power.shape)))

    inverse_shape = forward_shape


class SigmoidTransform(Transform):
    _type = Type.BIJECTION

    def _forward(self, x):
        return torch.sigmoid(x)

    def _inverse(self, y):
        return y.log() - (-y).log1p()

    def _forward_log_det_jacobian(self, x):
        return -TF.softplus(-x) - TF.softplus(x)


class TanhTransform(Transform):
    _type = Type.BIJECTION

    def _forward(self, x):
        return x.tanh()

    def _inverse(self, y):
        return torch.atanh(y)

    def _forward_log_det_jacobian(self, x):
        return 2.0 * (math.log(2.0) - x - TF.softplus(-2.0 * x))


class SoftmaxTransform(Transform):
    _type = Type.OTHER
    _domain = _Var(False, 1)
    _codomain = _Var(False, 1)

    def _forward(self, x):
        x = (x - x.max(-1, keepdim=True).values).exp()
        return x / x.sum(-1, keepdim=True)

    def _inverse(self, y):
        return y.log()

    def _forward_log_det_jacobian(self, x):
        raise NotImplementedError("SoftmaxTransform is not bijective")

    def forward_shape(self, shape):
        if len(shape) < 1:
            raise ValueError("SoftmaxTransform expects at least 1-D input")
        return tuple(shape)


class StickBreakingTransform(Transform):
    _type = Type.BIJECTION
    _domain = _Var(False, 1)
    _codomain = _Var(False, 1)

    def _forward(self, x):
        offset = x.shape[-1] + 1 - torch.ones([x.shape[-1]], device=x.device, dtype=x.dtype).cumsum(-1)
        z = torch.sigmoid(x - offset.log())
        z_cumprod = (1 - z).cumprod(-1)
        return TF.pad(z, [0, 1], value=1) * TF.pad(z_cumprod, [1, 0], value=1)

    def _inverse(self, y):
        y_crop = y[..., :-1]
        offset = y.shape[-1] - torch.ones([y_crop.shape[-1]], device=y.device, dtype=y.dtype).cumsum(-1)
        sf = 1 - y_crop.cumsum(-1)
        x = y_crop.log() - sf.log() + offset.log()
        return x

    def _forward_log_det_jacobian(self, x):
        y = self._forward(x)
        offset = x.shape[-1] + 1 - torch.ones([x.shape[-1]], device=x.device, dtype=x.dtype).cumsum(-1)
        x = x - offset.log()
        return (-x + TF.logsigmoid(x) + y[..., :-1].log()).sum(-1)

    def forward_shape(self, shape):
        return tuple(shape[:-1]) + (shape[-1] + 1,)

    def inverse_shape(self, shape):
        return tuple(shape[:-1]) + (shape[-1] - 1,)


class ReshapeTransform(Transform):
    _type = Type.BIJECTION

    def __init__(self, in_event_shape, out_event_shape):
        self.in_event_shape = tuple(in_event_shape)
        self.out_event_shape = tuple(out_event_shape)
        if functools.reduce(operator.mul, self.in_event_shape, 1) != functools.reduce(operator.mul,
                                                                                     self.out_event_shape, 1):
            raise ValueError("The numel of 'in_event_shape' should be 'out_event_shape'")
        self._domain = _Var(False, len(self.in_event_shape))
        self._codomain = _Var(False, len(self.out_event_shape))

    def _forward(self, x):
        return x.reshape(tuple(x.shape[:x.dim() - len(self.in_event_shape)]) + self.out_event_shape)

    def _inverse(self, y):
        return y.reshape(tuple(y.shape[:y.dim() - len(self.out_event_shape)]) + self.in_event_shape)

    def _forward_log_det_jacobian(self, x):
        return torch.zeros(x.shape[:x.dim() - len(self.in_event_shape)], dtype=x.dtype, device=x.device)

    def forward_shape(self, shape):
        n = len(self.in_event_shape)
        if tuple(shape[len(shape) - n:]) != self.in_event_shape:
            raise ValueError(f"Event shape mismatch, expected {self.in_event_shape}, got {shape}")
        return tuple(shape[:len(shape) - n]) + self.out_event_shape

    def inverse_shape(self, shape):
        n = len(self.out_event_shape)
        return tuple(shape[:len(shape) - n]) + self.in_event_shape


class IndependentTransform(Transform):
    def __init__(self, base, reinterpreted_batch_rank):
        if reinterpreted_batch_rank <= 0:
            raise ValueError("'reinterpreted_batch_rank' must be positive")
        self._base = base
        self._rank = reinterpreted_batch_rank
        self._type = base._type
        self._domain = _Var(base._domain.is_discrete, base._domain.event_rank + reinterpreted_batch_rank)
        self._codomain = _Var(base._codomain.is_discrete, base._codomain.event_rank + reinterpreted_batch_rank)

    def _forward(self, x):
        return self._base._forward(x)

    def _inverse(self, y):
        return self._base._inverse(y)

    def _forward_log_det_jacobian(self, x):
        return self._base._forward_log_det_jacobian(x).sum(tuple(range(-self._rank, 0)))

    def forward_shape(self, shape):
        return self._base.forward_shape(shape)

    def inverse_shape(self, shape):
        return self._base.inverse_shape(shape)


class ChainTransform(Transform):
    def __init__(self, transforms):
        if not all(isinstance(t, Transform) for t in transforms):
            raise TypeError("All elements of transforms should be Transform type")
        self.transforms = list(transforms)
        self._type = Type.BIJECTION if all(t._is_injective() for t in self.transforms) else Type.OTHER
        self._domain = _Var(False, max([t._domain.event_rank for t in self.transforms] or [0]))
        self._codomain = _Var(False, max([t._codomain.event_rank for t in self.transforms] or [0]))

    def _is_injective(self):
        return all(t._is_injective() for t in self.transforms)

    def _forward(self, x):
        for t in self.transforms:
            x = t._forward(x)
        return x

    def _inverse(self, y):
        for t in reversed(self.transforms):
            y = t._inverse(y)
        return y

    def _forward_log_det_jacobian(self, x):
        value = 0.0
        ev = self._domain.event_rank
        for t in self.transforms:
            ldj = t._forward_log_det_jacobian(x)
            extra = ev - t._domain.event_rank
            if extra > 0:
                ldj = ldj.sum(tuple(range(-extra, 0)))
            value = value + ldj
            x = t._forward(x)
            ev += t._codomain.event_rank - t._domain.event_rank
        return value

    def forward_shape(self, shape):
        for t in self.transforms:
            shape = t.forward_shape(shape)
        return tuple(shape)

    def inverse_shape(self, shape):
        for t in reversed(self.transforms):
            shape = t.inverse_shape(shape)
        return tuple(shape)


class StackTransform(Transform):
    def __init__(self, transforms, axis=0):
        if not transforms or not all(isinstance(t, Transform) for t in transforms):
            raise TypeError("Expected 'transforms' is Sequence[Transform]")
        self._transforms = list(transforms)
        self._axis = axis

    @property
    def transforms(self):
        return self._transforms

    @property
    def axis(self):
        return self._axis

    def _is_injective(self):
        return all(t._is_injective() for t in self._transforms)

    def _map(self, fn_name, v):
        parts = v.unbind(self._axis)
        if len(parts) != len(self._transforms):
            raise ValueError("Input dimensions mismatch the number of transforms")
        return torch.stack([getattr(t, fn_name)(p) for t, p in zip(self._transforms, parts)], self._axis)

    def _forward(self, x):
        return self._map("_forward", x)

    def _inverse(self, y):
        return self._map("_inverse", y)

    def _forward_log_det_jacobian(self, x):
        return self._map("_forward_log_det_jacobian", x)
