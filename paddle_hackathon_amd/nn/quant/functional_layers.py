"""Float functional ops as Layers (reference: python/paddle/nn/quant/functional_layers.py), so a
model that builds them as sublayers lets the quantization tools observe / fake-quant their
outputs (ImperativeQuantAware wraps them in output-scale layers)."""
from __future__ import annotations

from ... import tensor as T
from ..layer.layers import Layer

__all__ = ["FloatFunctionalLayer", "add", "subtract", "multiply", "divide", "reshape", "transpose", "concat",
           "flatten"]


class FloatFunctionalLayer(Layer):
    def __init__(self):
        super().__init__()


def _binary(name, fn):
    def forward(self, x, y, name=None):
        return fn(x, y)
    return type(name, (FloatFunctionalLayer,), {"forward": forward, "__doc__": f"``paddle.{name}`` as a Layer"})


add = _binary("add", T.add)
subtract = _binary("subtract", T.subtract)
multiply = _binary("multiply", T.multiply)
divide = _binary("divide", T.divide)


class reshape(FloatFunctionalLayer):
    def forward(self, x, shape, name=None):
        return T.reshape(x, shape)


class transpose(FloatFunctionalLayer):
    def forward(self, x, perm, name=None):
        return T.transpose(x, perm)


class concat(FloatFunctionalLayer):
    def forward(self, x, axis=0, name=None):
        return T.concat(x, axis)


class flatten(FloatFunctionalLayer):
    def forward(self, x, start_axis=0, stop_axis=-1, name=None):
        return T.flatten(x, start_axis, stop_axis)
