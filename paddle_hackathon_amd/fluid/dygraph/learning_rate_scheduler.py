"""``fluid.dygraph`` learning-rate decays (reference:
python/paddle/fluid/dygraph/learning_rate_scheduler.py). 1.x semantics: the schedule is a
function of ``step_num = begin + k * step`` where k counts optimizer steps — fluid optimizers
advance it after every ``minimize`` / ``step`` (fluid/optimizer.py) — and calling the object
returns the current rate. They are ``LRScheduler`` s, so the 2.x optimizers accept them too."""
from __future__ import annotations

import math

from ...optimizer.lr import LRScheduler

__all__ = ["LearningRateDecay", "NoamDecay", "PiecewiseDecay", "NaturalExpDecay", "ExponentialDecay",
           "InverseTimeDecay", "PolynomialDecay", "CosineDecay", "LinearLrWarmup", "ReduceLROnPlateau", "StepDecay",
           "MultiStepDecay", "LambdaDecay"]


class LearningRateDecay(LRScheduler):
    fluid_auto_step = True

    def __init__(self, begin=0, step=1, dtype="float32", learning_rate=1.0):
        self.begin, self.step_size, self.dtype = begin, step, dtype
        super().__init__(float(learning_rate))

    @property
    def step_num(self):
        return self.begin + self.last_epoch * self.step_size

    def get_lr(self):
        return float(self.lr_at(self.step_num))

    def lr_at(self, n):
        raise NotImplementedError


class NoamDecay(LearningRateDecay):
    def __init__(self, d_model, warmup_steps, begin=1, step=1, dtype="float32", learning_rate=1.0):
        self.d_model, self.warmup_steps = d_model, warmup_steps
        super().__init__(begin, step, dtype, learning_rate)

    def lr_at(self, n):
        n = max(n, 1)
        return self.base_lr * self.d_model ** -0.5 * min(n ** -0.5, self.warmup_steps ** -1.5 * n)


class PiecewiseDecay(LearningRateDecay):
    def __init__(self, boundaries, values, begin, step=1, dtype="float32"):
        self.boundaries, self.values = list(boundaries), list(values)
        super().__init__(begin, step, dtype, values[0])

    def lr_at(self, n):
        for b, v in zip(self.boundaries, self.values):
            if n < b:
                return v
        return self.values[len(self.boundaries)]


def _div(n, d, staircase):
    r = n / d
    return math.floor(r) if staircase else r


class NaturalExpDecay(LearningRateDecay):
    def __init__(self, learning_rate, decay_steps, decay_rate, staircase=False, begin=0, step=1, dtype="float32"):
        self.decay_steps, self.decay_rate, self.staircase = decay_steps, decay_rate, staircase
        super().__init__(begin, step, dtype, learning_rate)

    def lr_at(self, n):
        return self.base_lr * math.exp(-self.decay_rate * _div(n, self.decay_steps, self.staircase))


class ExponentialDecay(LearningRateDecay):
    def __init__(self, learning_rate, decay_steps, decay_rate, staircase=False, begin=0, step=1, dtype="float32"):
        self.decay_steps, self.decay_rate, self.staircase = decay_steps, decay_rate, staircase
        super().__init__(begin, step, dtype, learning_rate)

    def lr_at(self, n):
        return self.base_lr * self.decay_rate ** _div(n, self.decay_steps, self.staircase)


class InverseTimeDecay(LearningRateDecay):
    def __init__(self, learning_rate, decay_steps, decay_rate, staircase=False, begin=0, step=1, dtype="float32"):
        self.decay_steps, self.decay_rate, self.staircase = decay_steps, decay_rate, staircase
        super().__init__(begin, step, dtype, learning_rate)

    def lr_at(self, n):
        return self.base_lr / (1 + self.decay_rate * _div(n, self.decay_steps, self.staircase))


class PolynomialDecay(LearningRateDecay):
    def __init__(self, learning_rate, decay_steps, end_learning_rate=0.0001, power=1.0, cycle=False, begin=0, step=1,
                 dtype="float32"):
        self.decay_steps, self.end_lr, self.power, self.cycle = decay_steps, end_learning_rate, power, cycle
        super().__init__(begin, step, dtype, learning_rate)

    def lr_at(self, n):
        ds = self.decay_steps
        if self.cycle:
            div = math.ceil(n / ds) if n > 0 else 1
            ds = ds * max(div, 1)
        else:
            n = min(n, ds)
        return (self.base_lr - self.end_lr) * (1 - n / ds) ** self.power + self.end_lr


class CosineDecay(LearningRateDecay):
    def __init__(self, learning_rate, step_each_epoch, epochs, begin=0, step=1, dtype="float32"):
        self.step_each_epoch, self.epochs = step_each_epoch, epochs
        super().__init__(begin, step, dtype, learning_rate)

    def lr_at(self, n):
        epoch = math.floor(n / self.step_each_epoch)
        return self.base_lr * 0.5 * (math.cos(epoch * math.pi / self.epochs) + 1)


class LinearLrWarmup(LearningRateDecay):
    """linear start_lr -> end_lr over ``warmup_steps``, then ``learning_rate`` (a float or another
    decay, which keeps stepping)"""

    def __init__(self, learning_rate, warmup_steps, start_lr, end_lr, begin=1, step=1, dtype="float32"):
        self.inner = learning_rate if isinstance(learning_rate, LRScheduler) else None
        self.after = None if self.inner else float(learning_rate)
        self.warmup_steps, self.start_lr, self.end_lr = warmup_steps, start_lr, end_lr
        super().__init__(begin, step, dtype, start_lr)

    def lr_at(self, n):
        if n < self.warmup_steps:
            return self.start_lr + (self.end_lr - self.start_lr) * n / self.warmup_steps
        if self.inner is not None:
            return self.inner()
        return self.after

    def step(self, epoch=None):
        super().step(epoch)
        if self.inner is not None and self.step_num > self.warmup_steps:
            self.inner.step()


class ReduceLROnPlateau(LearningRateDecay):
    fluid_auto_step = False

    def __init__(self, learning_rate, mode="min", decay_rate=0.1, patience=10, verbose=False, threshold=1e-4,
                 threshold_mode="rel", cooldown=0, min_lr=0, eps=1e-8, dtype="float32"):
        self.mode, self.decay_rate, self.patience = mode, decay_rate, patience
        self.threshold, self.threshold_mode, self.cooldown = threshold, threshold_mode, cooldown
        self.min_lr, self.eps = min_lr, eps
        self.best, self.num_bad, self.cooldown_counter = None, 0, 0
        self.cur = float(learning_rate)
        super().__init__(0, 1, dtype, learning_rate)
        self.verbose = verbose

    def lr_at(self, n):
        return self.cur

    def _better(self, a, b):
        if self.threshold_mode == "rel":
            t = b * (1 - self.threshold) if self.mode == "min" else b * (1 + self.threshold)
        else:
            t = b - self.threshold if self.mode == "min" else b + self.threshold
        return a < t if self.mode == "min" else a > t

    def step(self, loss=None):
        if loss is None:
            return super().step()
        v = float(loss.numpy().reshape(-1)[0]) if hasattr(loss, "numpy") else float(loss)
        if self.best is None or self._better(v, self.best):
            self.best, self.num_bad = v, 0
        else:
            self.num_bad += 1
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
            self.num_bad = 0
        if self.num_bad > self.patience:
            new = max(self.cur * self.decay_rate, self.min_lr)
            if self.cur - new > self.eps:
                self.cur = new
            self.cooldown_counter, self.num_bad = self.cooldown, 0
        self.last_lr = self.cur
        self._push_device_lr()


class StepDecay(LearningRateDecay):
    fluid_auto_step = False     # epoch-based: the user calls epoch()

    def __init__(self, learning_rate, step_size, decay_rate=0.1):
        self.step_size_epochs, self.decay_rate = step_size, decay_rate
        super().__init__(0, 1, "float32", learning_rate)

    def epoch(self, epoch=None):
        self.step(epoch)

    def lr_at(self, n):
        return self.base_lr * self.decay_rate ** (n // self.step_size_epochs)


class MultiStepDecay(LearningRateDecay):
    fluid_auto_step = False

    def __init__(self, learning_rate, milestones, decay_rate=0.1):
        self.milestones, self.decay_rate = list(milestones), decay_rate
        super().__init__(0, 1, "float32", learning_rate)

    def epoch(self, epoch=None):
        self.step(epoch)

    def lr_at(self, n):
        k = sum(1 for m in self.milestones if n >= m)
        return self.base_lr * self.decay_rate ** k


class LambdaDecay(LearningRateDecay):
    fluid_auto_step = False

    def __init__(self, learning_rate, lr_lambda):
        self.lr_lambda = lr_lambda
        super().__init__(0, 1, "float32", learning_rate)

    def epoch(self, epoch=None):
        self.step(epoch)

    def lr_at(self, n):
        return self.base_lr * self.lr_lambda(n)
