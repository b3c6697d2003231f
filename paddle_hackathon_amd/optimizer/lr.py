"""Learning-rate schedulers (reference: python/paddle/optimizer/lr.py). Pure host
logic; the current LR is passed to the fused optimizer kernels as a scalar."""
from __future__ import annotations

import math
import warnings

import numpy as np

__all__ = ["LRScheduler", "NoamDecay", "PiecewiseDecay", "NaturalExpDecay", "InverseTimeDecay", "PolynomialDecay",
           "LinearWarmup", "ExponentialDecay", "MultiStepDecay", "StepDecay", "LambdaDecay", "ReduceOnPlateau",
           "CosineAnnealingDecay", "MultiplicativeDecay", "OneCycleLR", "CyclicLR"]


class LRScheduler:
    def __init__(self, learning_rate=0.1, last_epoch=-1, verbose=False):
        if not isinstance(learning_rate, (float, int)):
            raise TypeError(f"learning_rate must be float, got {type(learning_rate)}")
        self.base_lr = float(learning_rate)
        self.last_lr = float(learning_rate)
        self.last_epoch = last_epoch
        self.verbose = verbose
        self._var_name = None
        self.step()

    def __call__(self):
        return self.last_lr

    def step(self, epoch=None):
        if epoch is None:
            self.last_epoch += 1
            self.last_lr = self.get_lr()
        else:
            self.last_epoch = epoch
            self.last_lr = self._get_closed_form_lr() if hasattr(self, "_get_closed_form_lr") else self.get_lr()
        if self.verbose:
            print(f"Epoch {self.last_epoch}: {type(self).__name__} set learning rate to {self.last_lr}.")
        self._push_device_lr()

    # device copies of the current LR that hipGraph-captured optimizer steps read (optimizer
    # _lr_device): refreshed here, on the host, between replays
    def _register_device_lr(self, t):
        import weakref
        self.__dict__.setdefault("_dev_lrs", []).append(weakref.ref(t))

    def _push_device_lr(self):
        for r in self.__dict__.get("_dev_lrs", ()):
            t = r()
            if t is not None:
                t.fill_(float(self.last_lr))

    def state_keys(self):
        self.keys = ["last_epoch", "last_lr"]

    def state_dict(self):
        self.state_keys()
        out = {}
        for k in self.keys:
            v = self.__dict__[k]
            out[k] = v
        return out

    def set_state_dict(self, state_dict):
        self.state_keys()
        for k in self.keys:
            if k in state_dict:
                self.__dict__[k] = state_dict[k]
            else:
                raise RuntimeError(f"missing key {k} in LRScheduler state")

    set_dict = set_state_dict

    def get_lr(self):
        raise NotImplementedError


class NoamDecay(LRScheduler):
    def __init__(self, d_model, warmup_steps, learning_rate=1.0, last_epoch=-1, verbose=False):
        self.d_model, self.warmup_steps = d_model, warmup_steps
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        if self.last_epoch == 0:
            a = 1
        else:
            a = self.last_epoch ** -0.5
        b = self.warmup_steps ** -1.5 * self.last_epoch
        return self.base_lr * (self.d_model ** -0.5) * min(a, b)


class PiecewiseDecay(LRScheduler):
    def __init__(self, boundaries, values, last_epoch=-1, verbose=False):
        self.boundaries, self.values = boundaries, values
        super().__init__(last_epoch=last_epoch, verbose=verbose)

    def get_lr(self):
        for i, b in enumerate(self.boundaries):
            if self.last_epoch < b:
                return self.values[i]
        return self.values[len(self.values) - 1]


class NaturalExpDecay(LRScheduler):
    def __init__(self, learning_rate, gamma, last_epoch=-1, verbose=False):
        self.gamma = gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * math.exp(-1 * self.gamma * self.last_epoch)


class InverseTimeDecay(LRScheduler):
    def __init__(self, learning_rate, gamma, last_epoch=-1, verbose=False):
        self.gamma = gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr / (1 + self.gamma * self.last_epoch)


class PolynomialDecay(LRScheduler):
    def __init__(self, learning_rate, decay_steps, end_lr=0.0001, power=1.0, cycle=False, last_epoch=-1, verbose=False):
        self.decay_steps, self.end_lr, self.power, self.cycle = decay_steps, end_lr, power, cycle
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        tmp_epoch_num = self.last_epoch
        tmp_decay_steps = self.decay_steps
        if self.cycle:
            div_res = math.ceil(float(self.last_epoch) / float(self.decay_steps))
            if self.last_epoch == 0:
                div_res = 1
            tmp_decay_steps = self.decay_steps * div_res
        else:
            tmp_epoch_num = min(self.last_epoch, self.decay_steps)
        return (self.base_lr - self.end_lr) * ((1 - float(tmp_epoch_num) / float(tmp_decay_steps)) ** self.power) + self.end_lr


class LinearWarmup(LRScheduler):
    def __init__(self, learning_rate, warmup_steps, start_lr, end_lr, last_epoch=-1, verbose=False):
        self.learning_rate = learning_rate
        self.warmup_steps, self.start_lr, self.end_lr = warmup_steps, start_lr, end_lr
        super().__init__(start_lr if isinstance(learning_rate, LRScheduler) else (learning_rate if isinstance(learning_rate, (int, float)) else start_lr),
                         last_epoch, verbose)

    def state_dict(self):
        d = super().state_dict()
        if isinstance(self.learning_rate, LRScheduler):
            d["LinearWarmup_LR"] = self.learning_rate.state_dict()
        return d

    def set_state_dict(self, state_dict):
        super().set_state_dict(state_dict)
        if isinstance(self.learning_rate, LRScheduler) and "LinearWarmup_LR" in state_dict:
            self.learning_rate.set_state_dict(state_dict["LinearWarmup_LR"])

    def get_lr(self):
        if self.last_epoch < self.warmup_steps:
            return (self.end_lr - self.start_lr) * float(self.last_epoch) / float(self.warmup_steps) + self.start_lr
        if isinstance(self.learning_rate, LRScheduler):
            self.learning_rate.step(self.last_epoch - self.warmup_steps)
            return self.learning_rate()
        return self.learning_rate


class ExponentialDecay(LRScheduler):
    def __init__(self, learning_rate, gamma, last_epoch=-1, verbose=False):
        self.gamma = gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * (self.gamma ** self.last_epoch)


class MultiStepDecay(LRScheduler):
    def __init__(self, learning_rate, milestones, gamma=0.1, last_epoch=-1, verbose=False):
        self.milestones, self.gamma = milestones, gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        for i in range(len(self.milestones)):
            if self.last_epoch < self.milestones[i]:
                return self.base_lr * (self.gamma ** i)
        return self.base_lr * (self.gamma ** len(self.milestones))


class StepDecay(LRScheduler):
    def __init__(self, learning_rate, step_size, gamma=0.1, last_epoch=-1, verbose=False):
        self.step_size, self.gamma = step_size, gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * (self.gamma ** (self.last_epoch // self.step_size))


class LambdaDecay(LRScheduler):
    def __init__(self, learning_rate, lr_lambda, last_epoch=-1, verbose=False):
        self.lr_lambda = lr_lambda
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * self.lr_lambda(self.last_epoch)


class MultiplicativeDecay(LRScheduler):
    def __init__(self, learning_rate, lr_lambda, last_epoch=-1, verbose=False):
        self.lr_lambda = lr_lambda
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        if self.last_epoch > 0:
            return self.last_lr * self.lr_lambda(self.last_epoch)
        return self.base_lr


class ReduceOnPlateau(LRScheduler):
    def __init__(self, learning_rate, mode="min", factor=0.1, patience=10, threshold=1e-4, threshold_mode="rel",
                 cooldown=0, min_lr=0, epsilon=1e-8, verbose=False):
        if factor >= 1.0:
            raise ValueError("new_lr = origin_lr * gamma and gamma should be < 1.0.")
        self.mode, self.factor, self.patience = mode.lower(), factor, patience
        self.threshold, self.threshold_mode = threshold, threshold_mode.lower()
        self.cooldown, self.min_lr, self.epsilon = cooldown, min_lr, epsilon
        self.cooldown_counter = 0
        self.best = None
        self.num_bad_epochs = 0
        self.base_lr = float(learning_rate)
        self.last_lr = float(learning_rate)
        self.last_epoch = 0
        self.verbose = verbose
        self._var_name = None

    def state_keys(self):
        self.keys = ["cooldown_counter", "best", "num_bad_epochs", "last_epoch", "last_lr"]

    def step(self, metrics, epoch=None):
        if epoch is None:
            self.last_epoch += 1
        else:
            self.last_epoch = epoch
        if hasattr(metrics, "_t"):
            metrics = float(metrics._t.reshape(-1)[0])
        metrics = float(np.asarray(metrics).reshape(-1)[0])
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
        else:
            if self.best is None or self._is_better(metrics, self.best):
                self.best = metrics
                self.num_bad_epochs = 0
            else:
                self.num_bad_epochs += 1
            if self.num_bad_epochs > self.patience:
                self.cooldown_counter = self.cooldown
                self.num_bad_epochs = 0
                new_lr = max(self.last_lr * self.factor, self.min_lr)
                if self.last_lr - new_lr > self.epsilon:
                    self.last_lr = new_lr
                    if self.verbose:
                        print(f"Epoch {self.last_epoch}: ReduceOnPlateau set learning rate to {self.last_lr}.")
                    self._push_device_lr()

    def _is_better(self, current, best):
        if self.mode == "min" and self.threshold_mode == "rel":
            return current < best - best * self.threshold
        if self.mode == "min" and self.threshold_mode == "abs":
            return current < best - self.threshold
        if self.mode == "max" and self.threshold_mode == "rel":
            return current > best + best * self.threshold
        return current > best + self.threshold


class CosineAnnealingDecay(LRScheduler):
    def __init__(self, learning_rate, T_max, eta_min=0, last_epoch=-1, verbose=False):
        self.T_max, self.eta_min = T_max, float(eta_min)
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        if self.last_epoch == 0:
            return self.base_lr
        if (self.last_epoch - 1 - self.T_max) % (2 * self.T_max) == 0:
            return self.last_lr + (self.base_lr - self.eta_min) * (1 - math.cos(math.pi / self.T_max)) / 2
        return (1 + math.cos(math.pi * self.last_epoch / self.T_max)) / (
            1 + math.cos(math.pi * (self.last_epoch - 1) / self.T_max)) * (self.last_lr - self.eta_min) + self.eta_min

    def _get_closed_form_lr(self):
        return self.eta_min + (self.base_lr - self.eta_min) * (1 + math.cos(math.pi * self.last_epoch / self.T_max)) / 2


class OneCycleLR(LRScheduler):
    def __init__(self, max_learning_rate, total_steps, divide_factor=25.0, end_learning_rate=0.0001,
                 phase_pct=0.3, anneal_strategy="cos", three_phase=False, last_epoch=-1, verbose=False):
        self.total_steps = total_steps
        initial_lr = max_learning_rate / float(divide_factor)
        if three_phase:
            self._step_config = [0, float(phase_pct * total_steps) - 1, float(2 * phase_pct * total_steps) - 2, total_steps - 1]
            self._lr_config = [initial_lr, max_learning_rate, initial_lr, end_learning_rate]
        else:
            self._step_config = [0, float(phase_pct * total_steps) - 1, total_steps - 1]
            self._lr_config = [initial_lr, max_learning_rate, end_learning_rate]
        self._steps_size = [self._step_config[i + 1] - self._step_config[i] for i in range(len(self._step_config) - 1)]
        self._steps_size.insert(0, 1)
        self.anneal_func = self._cos_annealing if anneal_strategy == "cos" else self._linear_annealing
        super().__init__(initial_lr, last_epoch, verbose)

    def _cos_annealing(self, start_lr, end_lr, pct):
        return end_lr + (start_lr - end_lr) / 2.0 * (math.cos(math.pi * pct) + 1)

    def _linear_annealing(self, start_lr, end_lr, pct):
        return (end_lr - start_lr) * pct + start_lr

    def get_lr(self):
        current_step = self.last_epoch
        if current_step > self.total_steps:
            raise ValueError(f"Tried to step {current_step} times. Only {self.total_steps} allowed")
        for i, (end_step, step_size) in enumerate(zip(self._step_config[1:], self._steps_size[1:])):
            if current_step <= end_step or i == len(self._step_config) - 2:
                pct = (current_step - self._step_config[i]) / step_size
                return self.anneal_func(self._lr_config[i], self._lr_config[i + 1], pct)


class CyclicLR(LRScheduler):
    def __init__(self, base_learning_rate, max_learning_rate, step_size_up, step_size_down=None, mode="triangular",
                 exp_gamma=1.0, scale_fn=None, scale_mode="cycle", last_epoch=-1, verbose=False):
        step_size_down = step_size_up if step_size_down is None else step_size_down
        self.cycle_size = step_size_up + step_size_down
        self.step_up_pct = step_size_up / self.cycle_size
        self.max_lr = float(max_learning_rate)
        self.amplitude = self.max_lr - base_learning_rate
        self.mode, self.gamma = mode, exp_gamma
        if scale_fn is None:
            if mode == "triangular":
                self.scale_fn, self.scale_mode = (lambda x: 1.0), "cycle"
            elif mode == "triangular2":
                self.scale_fn, self.scale_mode = (lambda x: 1 / (2.0 ** (x - 1))), "cycle"
            else:
                self.scale_fn, self.scale_mode = (lambda x: self.gamma ** x), "iterations"
        else:
            self.scale_fn, self.scale_mode = scale_fn, scale_mode
        super().__init__(base_learning_rate, last_epoch, verbose)

    def get_lr(self):
        iterations = self.last_epoch
        cycle = 1 + iterations // self.cycle_size
        pct = 1.0 + iterations / self.cycle_size - cycle
        if pct <= self.step_up_pct:
            scale_factor = pct / self.step_up_pct
        else:
            scale_factor = (1 - pct) / (1 - self.step_up_pct)
        base_height = self.amplitude * scale_factor
        x = cycle if self.scale_mode == "cycle" else iterations
        return self.base_lr + base_height * self.scale_fn(x)
