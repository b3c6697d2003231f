"""``WeightedAverage`` (reference: python/paddle/fluid/average.py)."""
import numpy as np

__all__ = ["WeightedAverage"]


class WeightedAverage:
    def __init__(self):
        self.reset()

    def reset(self):
        self.numerator = None
        self.denominator = None

    def add(self, value, weight):
        v = np.asarray(value, dtype="float64")
        w = float(np.asarray(weight).reshape(-1)[0]) if np.ndim(weight) else float(weight)
        if self.numerator is None:
            self.numerator, self.denominator = v * w, w
        else:
            self.numerator = self.numerator + v * w
            self.denominator += w

    def eval(self):
        if self.numerator is None:
            raise ValueError("There is no data to be averaged in WeightedAverage.")
        return self.numerator / self.denominator
