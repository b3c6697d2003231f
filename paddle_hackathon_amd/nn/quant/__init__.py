"""``paddle.nn.quant`` (reference: python/paddle/nn/quant/__init__.py): quantization-aware layers,
float functional layers and the fake-quant ops (HIP kernels: csrc/kernels/quant.hip)."""
from .functional_layers import FloatFunctionalLayer, add, subtract, multiply, divide, reshape, transpose, \
    concat, flatten  # noqa: F401
from .quant_layers import QuantStub, FakeQuantAbsMax, FakeQuantMovingAverageAbsMax, \
    FakeQuantChannelWiseAbsMax, MovingAverageAbsMaxScale, QuantizedConv2D, QuantizedConv2DTranspose, \
    QuantizedLinear, MAOutputScaleLayer, FakeQuantMAOutputScaleLayer  # noqa: F401
from . import quant_layers, functional_layers, ops  # noqa: F401

__all__ = []
