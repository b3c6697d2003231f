"""incubate optimizers (reference: python/paddle/incubate/optimizer/{lookahead,modelaverage,
distributed_fused_lamb}.py, functional/{bfgs,lbfgs}.py)."""
from __future__ import annotations

import torch

from ...framework.core import Tensor, _wrap
from ...optimizer.optimizer import Optimizer, Lamb
from . import functional  # noqa: F401

__all__ = ["LookAhead", "ModelAverage", "DistributedFusedLamb"]


class LookAhead(Optimizer):
    """Every ``k`` inner steps: slow = slow + alpha * (fast - slow); fast = slow."""

    def __init__(self, inner_optimizer, alpha=0.5, k=5, name=None):
        if inner_optimizer is None:
            raise ValueError("inner optimizer can not be None")
        if not 0.0 <= alpha <= 1.0:
            raise ValueError("alpha should be in [0.0, 1.0]")
        if not (isinstance(k, int) and k > 0):
            raise ValueError("k should be a positive integer")
        self.inner_optimizer = inner_optimizer
        self.alpha, self.k = alpha, k
        self._parameter_list = inner_optimizer._parameter_list
        self._param_groups = inner_optimizer._param_groups
        self._learning_rate = inner_optimizer._learning_rate
        self._grad_clip = None
        self._name = name
        self._slow = {}
        self._global_step = 0
        self._accumulators = inner_optimizer._accumulators
        self._master_weights = inner_optimizer._master_weights
        self._state_loaded = {}
        self._step_count = 0

    @torch.no_grad()
    def step(self):
        self.inner_optimizer.step()
        self._global_step += 1
        params = [p for p in self._parameter_list if not p.stop_gradient]
        if self._global_step == 1:
            for p in params:
                self._slow[p.name] = p._t.detach().clone()
        if self._global_step % self.k == 0:
            for p in params:
                slow = self._slow.setdefault(p.name, p._t.detach().clone())
                slow.add_(p._t - slow, alpha=self.alpha)
                p._t.copy_(slow)

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        loss.backward()
        self.step()
        return None, None

    def clear_grad(self, set_to_zero=True):
        self.inner_optimizer.clear_grad(set_to_zero)

    def state_dict(self):
        sd = self.inner_optimizer.state_dict()
        for k, v in self._slow.items():
            sd[f"{k}@SLOW"] = _wrap(v)
        sd["@LOOKAHEAD_STEP"] = self._global_step
        return sd

    def set_state_dict(self, state):
        state = dict(state)
        self._global_step = int(state.pop("@LOOKAHEAD_STEP", 0))
        for k in [k for k in state if k.endswith("@SLOW")]:
            v = state.pop(k)
            self._slow[k[:-5]] = (v._t if isinstance(v, Tensor) else torch.as_tensor(v)).clone()
        self.inner_optimizer.set_state_dict(state)


class ModelAverage(Optimizer):
    """Sliding-window parameter averaging (reference modelaverage.py): keeps sum_1/sum_2/sum_3
    accumulators; ``apply()`` swaps in the average, ``restore()`` swaps back."""

    def __init__(self, average_window_rate, parameters=None, min_average_window=10000, max_average_window=10000,
                 name=None):
        super().__init__(learning_rate=0.0, parameters=parameters, name=name)
        self.average_window = average_window_rate
        self.min_average_window, self.max_average_window = min_average_window, max_average_window
        self._state = {}
        self._backup = {}

    def _st(self, p):
        s = self._state.get(p.name)
        if s is None:
            z = torch.zeros_like(p._t, dtype=torch.float32)
            s = self._state[p.name] = {"sum_1": z.clone(), "sum_2": z.clone(), "sum_3": z.clone(),
                                       "num_accumulates": 0, "old_num_accumulates": 0, "num_updates": 0}
        return s

    @torch.no_grad()
    def step(self):
        for p in self._parameter_list:
            if p.stop_gradient:
                continue
            s = self._st(p)
            s["num_updates"] += 1
            s["num_accumulates"] += 1
            s["sum_1"].add_(p._t.float())
            if s["num_updates"] % 16384 == 0:  # fold into sum_2 to bound fp32 error (reference kMaxNumAccumulates)
                s["sum_2"].add_(s["sum_1"])
                s["sum_1"].zero_()
            window = min(self.max_average_window, s["num_updates"] * self.average_window)
            if s["num_accumulates"] >= self.min_average_window and s["num_accumulates"] >= window:
                s["sum_3"].copy_(s["sum_1"] + s["sum_2"])
                s["sum_1"].zero_()
                s["sum_2"].zero_()
                s["old_num_accumulates"] = s["num_accumulates"]
                s["num_accumulates"] = 0

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        self.step()
        return None, None

    @torch.no_grad()
    def apply(self, executor=None, need_restore=True):
        import contextlib

        for p in self._parameter_list:
            s = self._state.get(p.name)
            if s is None:
                continue
            n = s["num_accumulates"] + s["old_num_accumulates"]
            if n == 0:
                continue
            self._backup[p.name] = p._t.detach().clone()
            p._t.copy_(((s["sum_1"] + s["sum_2"] + s["sum_3"]) / n).to(p._t.dtype))

        @contextlib.contextmanager
        def guard():
            try:
                yield
            finally:
                if need_restore:
                    self.restore()
        return guard()

    @torch.no_grad()
    def restore(self, executor=None):
        for p in self._parameter_list:
            b = self._backup.pop(p.name, None)
            if b is not None:
                p._t.copy_(b)


from .distributed_fused_lamb import DistributedFusedLamb  # noqa: E402,F401
