"""``paddle.tensor.stat`` (reference: python/paddle/tensor/stat.py)."""
from .. import mean, std, var, median, quantile, numel  # noqa: F401

__all__ = ["mean", "std", "var", "median", "quantile", "numel"]
