"""``paddle.fluid.initializer`` (reference: python/paddle/fluid/initializer.py): 1.x names and
signatures over the framework initializers."""
from __future__ import annotations

from ..nn import initializer as _I
from ..nn.initializer import (Constant, Bilinear, NumpyArrayInitializer, set_global_initializer,  # noqa: F401
                              ConstantInitializer, Initializer)

__all__ = ["Constant", "Uniform", "Normal", "TruncatedNormal", "Xavier", "Bilinear", "MSRA", "ConstantInitializer",
           "UniformInitializer", "NormalInitializer", "TruncatedNormalInitializer", "XavierInitializer",
           "BilinearInitializer", "MSRAInitializer", "NumpyArrayInitializer", "set_global_initializer"]


class UniformInitializer(_I.Uniform):
    def __init__(self, low=-1.0, high=1.0, seed=0, diag_num=0, diag_step=0, diag_val=1.0):
        super().__init__(low, high)


class NormalInitializer(_I.Normal):
    def __init__(self, loc=0.0, scale=1.0, seed=0):
        super().__init__(loc, scale)


class TruncatedNormalInitializer(_I.TruncatedNormal):
    def __init__(self, loc=0.0, scale=1.0, seed=0):
        super().__init__(loc, scale)


class XavierInitializer(_I.Initializer):
    """uniform (default) or normal Xavier / Glorot"""

    def __init__(self, uniform=True, fan_in=None, fan_out=None, seed=0):
        self._impl = _I.XavierUniform(fan_in, fan_out) if uniform else _I.XavierNormal(fan_in, fan_out)

    def __call__(self, param, block=None):
        return self._impl(param, block)


class MSRAInitializer(_I.Initializer):
    """Kaiming / He (uniform by default, like 1.x)"""

    def __init__(self, uniform=True, fan_in=None, seed=0, negative_slope=0.0, nonlinearity="relu"):
        self._impl = _I.KaimingUniform(fan_in, negative_slope, nonlinearity) if uniform else \
            _I.KaimingNormal(fan_in, negative_slope, nonlinearity)

    def __call__(self, param, block=None):
        return self._impl(param, block)


BilinearInitializer = Bilinear
Uniform = UniformInitializer
Normal = NormalInitializer
TruncatedNormal = TruncatedNormalInitializer
Xavier = XavierInitializer
MSRA = MSRAInitializer
