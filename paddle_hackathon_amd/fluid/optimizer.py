"""``paddle.fluid.optimizer`` (reference: python/paddle/fluid/optimizer.py).

The 1.x optimizers take ``parameter_list`` / ``regularization`` and, in dygraph mode, apply the
gradients already produced by ``loss.backward()`` when ``minimize(loss)`` is called. They are
the framework optimizers (fused multi-tensor HIP updates for Momentum / Adam) under their 1.x
constructor signatures, plus the 1.x-only rules (DecayedAdagrad, Ftrl, Dpsgd) and wrappers
(ModelAverage, ExponentialMovingAverage, Lookahead, Recompute, Pipeline). A ``fluid.dygraph``
learning-rate decay advances once per minimize.
"""
from __future__ import annotations

import torch

from ..framework import core as _core
from .. import optimizer as _O
from ..optimizer.optimizer import Optimizer as _Base
from ..incubate.optimizer import LookAhead as _LookAhead, ModelAverage as _ModelAverage
from ..parallel.fleet.meta_optimizers import LarsMomentumOptimizer as _Lars
from ..static import ExponentialMovingAverage  # noqa: F401

__all__ = ["SGD", "Momentum", "Adagrad", "Adam", "Adamax", "Dpsgd", "DecayedAdagrad", "Ftrl", "SGDOptimizer",
           "MomentumOptimizer", "AdagradOptimizer", "AdamOptimizer", "AdamaxOptimizer", "DpsgdOptimizer",
           "DecayedAdagradOptimizer", "RMSPropOptimizer", "FtrlOptimizer", "Adadelta", "AdadeltaOptimizer",
           "ModelAverage", "LarsMomentum", "LarsMomentumOptimizer", "LambOptimizer", "ExponentialMovingAverage",
           "PipelineOptimizer", "LookaheadOptimizer", "RecomputeOptimizer"]


class _Fluid:
    """1.x behaviour mixed into a framework optimizer class"""

    def _fluid_after_step(self):
        lr = self._learning_rate
        if getattr(lr, "fluid_auto_step", False):
            lr.step()

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        if not _core.in_dynamic_mode():
            from ..static.program import minimize_static
            return minimize_static(self, loss, parameter_list, no_grad_set)
        if parameter_list is not None and self._parameter_list is None:
            self._add_param_group({"params": list(parameter_list)})
            self._parameter_list = list(parameter_list)
        self.step()
        self._fluid_after_step()
        return None, [(p, p.grad) for p in (self._parameter_list or []) if p._t.grad is not None]

    def clear_gradients(self):
        self.clear_grad(set_to_zero=False)

    def current_step_lr(self):
        return self.get_lr()

    def set_dict(self, state_dict):
        self.set_state_dict(state_dict)


def _fluid(base, extra_init=None):
    def __init__(self, learning_rate, *args, parameter_list=None, regularization=None, grad_clip=None, name=None,
                 **kw):
        kw = {k: v for k, v in kw.items() if k not in ("lazy_mode",)}
        base.__init__(self, learning_rate, *args, parameters=parameter_list, weight_decay=regularization,
                      grad_clip=grad_clip, name=name, **kw)
    return type(base.__name__, (_Fluid, base), {"__init__": __init__, "__doc__": base.__doc__})


SGDOptimizer = _fluid(_O.SGD)
MomentumOptimizer = _fluid(_O.Momentum)
AdagradOptimizer = _fluid(_O.Adagrad)
AdamaxOptimizer = _fluid(_O.Adamax)
AdadeltaOptimizer = _fluid(_O.Adadelta)
RMSPropOptimizer = _fluid(_O.RMSProp)


class AdamOptimizer(_Fluid, _O.Adam):
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameter_list=None,
                 regularization=None, grad_clip=None, name=None, lazy_mode=False, multi_precision=False, **kw):
        _O.Adam.__init__(self, learning_rate, beta1, beta2, epsilon, parameters=parameter_list,
                         weight_decay=regularization, grad_clip=grad_clip, name=name, lazy_mode=lazy_mode,
                         multi_precision=multi_precision)


class LambOptimizer(_Fluid, _O.Lamb):
    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999, epsilon=1e-6,
                 parameter_list=None, regularization=None, grad_clip=None, exclude_from_weight_decay_fn=None,
                 name=None):
        _O.Lamb.__init__(self, learning_rate, lamb_weight_decay, beta1, beta2, epsilon, parameters=parameter_list,
                         grad_clip=grad_clip, exclude_from_weight_decay_fn=exclude_from_weight_decay_fn, name=name)


class LarsMomentumOptimizer(_Fluid, _Lars):
    def __init__(self, learning_rate, momentum, lars_coeff=0.001, lars_weight_decay=0.0005, parameter_list=None,
                 regularization=None, grad_clip=None, name=None, exclude_from_weight_decay=None, epsilon=0,
                 multi_precision=False, rescale_grad=1.0):
        _Lars.__init__(self, learning_rate, momentum, lars_coeff, lars_weight_decay, parameters=parameter_list,
                       grad_clip=grad_clip, exclude_from_weight_decay=exclude_from_weight_decay, epsilon=epsilon,
                       multi_precision=multi_precision, rescale_grad=rescale_grad, name=name)


class DecayedAdagradOptimizer(_Fluid, _Base):
    """moment = decay * moment + (1 - decay) * g^2; p -= lr * g / (sqrt(moment) + eps)"""

    def __init__(self, learning_rate, decay=0.95, epsilon=1.0e-6, parameter_list=None, regularization=None,
                 grad_clip=None, name=None):
        _Base.__init__(self, learning_rate, parameter_list, regularization, grad_clip, name, False)
        self._decay, self._epsilon = decay, epsilon

    def _update(self, pgs):
        lr = self.get_lr()
        for p, g, group in pgs:
            wd, kind = self._wd_for(p, group)
            gt = g._t.float() + (wd * p._t.float() if kind == "l2" else 0)
            m = self._acc("moment", p)._t
            m.mul_(self._decay).add_(gt * gt, alpha=1 - self._decay)
            p._t.sub_((lr * self._lr_ratio(p, group) * gt / (m.sqrt() + self._epsilon)).to(p._t.dtype))


class FtrlOptimizer(_Fluid, _Base):
    """FTRL-proximal (ftrl_op.h) with l1 / l2 regularisation and learning-rate power"""

    def __init__(self, learning_rate, l1=0.0, l2=0.0, lr_power=-0.5, parameter_list=None, regularization=None,
                 grad_clip=None, name=None):
        _Base.__init__(self, learning_rate, parameter_list, regularization, grad_clip, name, False)
        self._l1, self._l2, self._lr_power = l1, l2, lr_power

    def _update(self, pgs):
        lr = self.get_lr()
        for p, g, group in pgs:
            gt = g._t.float()
            w = p._t.float()
            sq = self._acc("squared", p)._t
            lin = self._acc("linear", p)._t
            lr_p = lr * self._lr_ratio(p, group)
            new_sq = sq + gt * gt
            if self._lr_power == -0.5:
                lin.add_(gt - (new_sq.sqrt() - sq.sqrt()) / lr_p * w)
                y = new_sq.sqrt() / lr_p + 2 * self._l2
            else:
                lin.add_(gt - (new_sq.pow(-self._lr_power) - sq.pow(-self._lr_power)) / lr_p * w)
                y = new_sq.pow(-self._lr_power) / lr_p + 2 * self._l2
            x = self._l1 * torch.sign(lin) - lin
            p._t.copy_(torch.where(lin.abs() > self._l1, x / y, torch.zeros_like(x)).to(p._t.dtype))
            sq.copy_(new_sq)


class DpsgdOptimizer(_Fluid, _Base):
    """differentially private SGD: per-step gradient clipped to L2 norm ``clip`` plus Gaussian noise
    of std ``sigma * clip`` averaged over ``batch_size`` (dpsgd_op.h)"""

    def __init__(self, learning_rate=0.001, clip=0.9, batch_size=0.999, sigma=1e-8, parameter_list=None,
                 seed=0):
        _Base.__init__(self, learning_rate, parameter_list, None, None, None, False)
        self._clip, self._batch, self._sigma = clip, batch_size, sigma
        self._gen = torch.Generator()
        if seed:
            self._gen.manual_seed(int(seed))

    def _update(self, pgs):
        lr = self.get_lr()
        for p, g, group in pgs:
            gt = g._t.float()
            n = float(gt.norm())
            scale = n / self._clip if n > self._clip else 1.0
            noise = torch.randn(gt.shape, generator=self._gen).to(gt.device) * self._sigma * self._clip
            p._t.sub_((lr * (gt / scale + noise / self._batch)).to(p._t.dtype))


SGD = SGDOptimizer
Momentum = MomentumOptimizer
Adagrad = AdagradOptimizer
Adam = AdamOptimizer
Adamax = AdamaxOptimizer
Dpsgd = DpsgdOptimizer
DecayedAdagrad = DecayedAdagradOptimizer
Ftrl = FtrlOptimizer
Adadelta = AdadeltaOptimizer
LarsMomentum = LarsMomentumOptimizer


class ModelAverage(_ModelAverage):
    def __init__(self, average_window_rate, min_average_window=10000, max_average_window=10000,
                 regularization=None, name=None, parameter_list=None):
        super().__init__(average_window_rate, parameter_list, min_average_window, max_average_window, name)


class LookaheadOptimizer(_LookAhead):
    def __init__(self, inner_optimizer, alpha=0.5, k=5):
        super().__init__(inner_optimizer, alpha, k)


class RecomputeOptimizer:
    """wraps an optimizer; ``_set_checkpoints`` names the recompute segment boundaries. Static
    mode inserts the recompute pass (static/passes.py recompute_segments); dygraph mode has the
    model decide with ``paddle.distributed.fleet.utils.recompute``."""

    def __init__(self, optimizer):
        self._optimizer = optimizer
        self._checkpoints = None

    def _set_checkpoints(self, checkpoints):
        self._checkpoints = list(checkpoints)

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        if _core.in_dynamic_mode():
            return self._optimizer.minimize(loss, startup_program, parameter_list, no_grad_set)
        from ..static.backward import append_backward
        from ..static.backward import append_optimize_op
        pg = append_backward(loss, parameter_list, no_grad_set, checkpoints=self._checkpoints)
        return append_optimize_op(self._optimizer, pg), pg

    def __getattr__(self, item):
        return getattr(self._optimizer, item)


class PipelineOptimizer:
    """1.x static pipeline: the program's ``device_guard("gpu:k")`` sections become stages, one
    per rank, run over ``num_microbatches`` micro-batches with point-to-point activation and
    gradient transfers (parallel/fleet/static_pipeline.py). Dygraph pipelines use
    fleet.meta_parallel.PipelineLayer (parallel/pipeline.py)."""

    def __init__(self, optimizer, num_microbatches=1, start_cpu_core_id=0):
        from ..parallel.fleet.static_pipeline import PipelineOptimizer as _P
        self._impl = _P(optimizer, num_microbatches)
        self._optimizer = optimizer

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        if _core.in_dynamic_mode():
            return self._optimizer.minimize(loss, startup_program, parameter_list, no_grad_set)
        return self._impl.minimize(loss, startup_program, parameter_list, no_grad_set)

    def __getattr__(self, item):
        return getattr(self._optimizer, item)
