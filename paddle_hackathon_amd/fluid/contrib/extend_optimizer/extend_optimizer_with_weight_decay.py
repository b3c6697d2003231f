"""``extend_with_decoupled_weight_decay`` (reference python/paddle/fluid/contrib/extend_optimizer/
extend_optimizer_with_weight_decay.py:101): an optimizer class whose update first decays the
parameters it updates, ``param -= param * coeff`` (the reference's scale / elementwise_sub /
assign ops in front of the optimizer ops), then applies the base optimizer's rule with the
gradients computed at the undecayed parameters. ``apply_decay_param_fun(name)`` selects the
parameters; ``coeff`` may be a float or a [1] tensor. The decay runs inside ``step``: in dygraph
from ``step`` / ``minimize``, in a static Program from the recorded optimizer op (which steps the
optimizer), so it precedes the update in both."""
from __future__ import annotations

import torch

from ....framework.core import Tensor
from ....optimizer.optimizer import Optimizer

__all__ = ["extend_with_decoupled_weight_decay", "DecoupledWeightDecay"]


class DecoupledWeightDecay:
    def __init__(self, coeff=0.0, apply_decay_param_fun=None, **kwargs):
        if not isinstance(coeff, (float, Tensor)):
            raise TypeError("coeff should be float or Variable.")
        self._params_name = set()
        self._apply_decay_param_fun = apply_decay_param_fun
        self._coeff = coeff
        super().__init__(**kwargs)

    def _decay_selected(self, params):
        return [p for p in params if self._apply_decay_param_fun is None or self._apply_decay_param_fun(p.name)]

    def _coeff_value(self):
        c = self._coeff
        return float(c._t.reshape(-1)[0]) if isinstance(c, Tensor) else float(c)

    def _decay(self, params):
        c = self._coeff_value()
        if c == 0.0:
            return
        with torch.no_grad():
            for p in self._decay_selected(params):
                self._params_name.add(p.name)
                p._t.mul_(1.0 - c)

    def step(self):
        self._decay([p for g in self._param_groups for p in g["params"] if p._t.grad is not None])
        return super().step()

    def __str__(self):
        return " ".join(["Weight Decay, params:", ",".join(sorted(self._params_name))])


def extend_with_decoupled_weight_decay(base_optimizer):
    """``OptimizerWithDecoupledWeightDecay(weight_decay, apply_decay_param_fun=None, **base kwargs)``"""
    if not (isinstance(base_optimizer, type) and issubclass(base_optimizer, Optimizer)):
        raise TypeError("The input(base_optimizer) should be a derived class of Optimizer.")

    class OptimizerWithDecoupledWeightDecay(DecoupledWeightDecay, base_optimizer):
        def __init__(self, weight_decay, apply_decay_param_fun=None, **kwargs):
            super().__init__(weight_decay, apply_decay_param_fun, **kwargs)

    OptimizerWithDecoupledWeightDecay.__name__ = "OptimizerWithDecoupledWeightDecay"
    return OptimizerWithDecoupledWeightDecay
