"""``fluid.layers`` learning-rate decay builders (reference:
python/paddle/fluid/layers/learning_rate_scheduler.py). Each returns the matching
``fluid.dygraph`` decay object (an ``LRScheduler``), which the fluid optimizers advance once per
optimisation step in both execution modes."""
from __future__ import annotations

from ..dygraph import learning_rate_scheduler as D

__all__ = ["exponential_decay", "natural_exp_decay", "inverse_time_decay", "polynomial_decay", "piecewise_decay",
           "noam_decay", "cosine_decay", "linear_lr_warmup"]


def noam_decay(d_model, warmup_steps, learning_rate=1.0):
    return D.NoamDecay(d_model, warmup_steps, learning_rate=learning_rate)


def exponential_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    return D.ExponentialDecay(learning_rate, decay_steps, decay_rate, staircase)


def natural_exp_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    return D.NaturalExpDecay(learning_rate, decay_steps, decay_rate, staircase)


def inverse_time_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    return D.InverseTimeDecay(learning_rate, decay_steps, decay_rate, staircase)


def polynomial_decay(learning_rate, decay_steps, end_learning_rate=0.0001, power=1.0, cycle=False):
    return D.PolynomialDecay(learning_rate, decay_steps, end_learning_rate, power, cycle)


def piecewise_decay(boundaries, values):
    return D.PiecewiseDecay(boundaries, values, 0)


def cosine_decay(learning_rate, step_each_epoch, epochs):
    return D.CosineDecay(learning_rate, step_each_epoch, epochs)


def linear_lr_warmup(learning_rate, warmup_steps, start_lr, end_lr):
    return D.LinearLrWarmup(learning_rate, warmup_steps, start_lr, end_lr, begin=0)
