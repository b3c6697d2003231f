"""Weight-decay regularizers (reference: python/paddle/regularizer.py).
Applied inside the fused optimizer kernels as an extra term on the gradient."""
from __future__ import annotations

__all__ = ["L1Decay", "L2Decay", "WeightDecayRegularizer"]


class WeightDecayRegularizer:
    coeff = 0.0


class L1Decay(WeightDecayRegularizer):
    def __init__(self, coeff=0.0):
        self.coeff = float(coeff)

    def __call__(self, param, grad):
        return grad + self.coeff * param.sign()


class L2Decay(WeightDecayRegularizer):
    def __init__(self, coeff=0.0):
        self.coeff = float(coeff)

    def __call__(self, param, grad):
        return grad + self.coeff * param


L1DecayRegularizer = L1Decay
L2DecayRegularizer = L2Decay
