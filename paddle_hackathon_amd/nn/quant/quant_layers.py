"""Quantization-aware-training layers (reference: python/paddle/nn/quant/quant_layers.py:47-746).

Fake-quant layers hold their scales as non-trainable parameters (so they are saved with the
model's state dict and written into exported programs) and call the fake-quant ops of
nn/quant/ops.py (HIP kernels on the GPU, straight-through gradients).

* ``FakeQuantAbsMax`` — per-tensor abs-max quant-dequant (weights: ``quant_on_weight`` keeps the
  last scale in a parameter)
* ``FakeQuantMovingAverageAbsMax`` — activations: scale = moving average of max |x| in training,
  the stored scale at eval
* ``FakeQuantChannelWiseAbsMax`` — per-output-channel weights (conv axis 0, linear axis 1)
* ``MovingAverageAbsMaxScale`` — output-scale observer (x passes through)
* ``QuantizedConv2D`` / ``QuantizedConv2DTranspose`` / ``QuantizedLinear`` — wrap a float layer:
  quantize its input and weight, then run the float op
* ``MAOutputScaleLayer`` / ``FakeQuantMAOutputScaleLayer`` — output observers around a layer
* ``QuantStub`` — marks a model input for quantization
"""
from __future__ import annotations

import torch

from ...framework.core import _wrap
from ...framework.param_attr import ParamAttr
from .. import functional as F
from ..initializer import Constant
from ..layer.layers import Layer
from . import ops as QO

__all__ = ["FakeQuantAbsMax", "FakeQuantMovingAverageAbsMax", "FakeQuantChannelWiseAbsMax", "MovingAverageAbsMaxScale",
           "QuantizedConv2D", "QuantizedConv2DTranspose", "QuantizedLinear", "MAOutputScaleLayer",
           "FakeQuantMAOutputScaleLayer", "QuantStub"]


def _unique(prefix):
    from ...utils import unique_name
    return unique_name.generate(prefix)


class _ScaleHolder(Layer):
    def _state_param(self, name, shape, value):
        p = self.create_parameter(list(shape), attr=ParamAttr(name=_unique(name), initializer=Constant(value),
                                                             trainable=False), dtype="float32")
        p.stop_gradient = True
        return p


class FakeQuantAbsMax(_ScaleHolder):
    """scale = max|X|, range = 2^(bits-1) - 1, Out = round(X / scale * range) * scale / range"""

    def __init__(self, name=None, quant_bits=8, dtype="float32", quant_on_weight=False, round_type=1):
        super().__init__()
        self._quant_bits = quant_bits
        self._name = name
        self._round_type = round_type
        self._scale_name = f"{name}.scale" if name else "quant_dequant.scale"
        self._scale = self._state_param(self._scale_name, [1], 0.001) if quant_on_weight else None

    def forward(self, input):
        out, scale = QO.fake_quantize_dequantize_abs_max(input, self._quant_bits, self._round_type)
        if self._scale is not None and not _is_meta(scale):
            with torch.no_grad():
                self._scale._t.copy_(scale._t.reshape(self._scale._t.shape))
        return out


def _is_meta(t):
    return getattr(t, "_t", t).device.type == "meta" or type(t).__name__ == "Variable"


class FakeQuantMovingAverageAbsMax(_ScaleHolder):
    """training: scale = accum / state with state = r*state + 1, accum = r*accum + max|X|;
    eval (``layer.eval()``): the stored scale"""

    def __init__(self, name=None, moving_rate=0.9, quant_bits=8, dtype="float32", round_type=1):
        super().__init__()
        self._moving_rate = moving_rate
        self._quant_bits = quant_bits
        self._round_type = round_type
        prefix = f"{name}.quant_dequant" if name else "quant_dequant"
        self._scale = self._state_param(prefix + ".scale", [1], 0.001)
        self._state = self._state_param(prefix + ".state", [1], 1.0)
        self._accum = self._state_param(prefix + ".accum", [1], 1.0)

    def forward(self, input):
        return QO.fake_quantize_dequantize_moving_average_abs_max(
            input, self._scale, self._state, self._accum, self._quant_bits, self._moving_rate, not self.training,
            self._round_type)


class FakeQuantChannelWiseAbsMax(_ScaleHolder):
    """per-channel abs-max quant-dequant along ``quant_axis``"""

    def __init__(self, name=None, channel_num=None, quant_bits=8, quant_axis=0, dtype="float32",
                 quant_on_weight=False, round_type=1):
        assert quant_on_weight, "Channel-wise quantization can only be used on weight"
        super().__init__()
        self._quant_bits = quant_bits
        self._quant_axis = quant_axis
        self._channel_num = channel_num
        self._round_type = round_type
        self._name = name
        self._scale_name = f"{name}.scale" if name else "quant_dequant.scale"
        self._scale = self._state_param(self._scale_name, [channel_num], 0.0)

    def forward(self, input):
        out, scale = QO.fake_channel_wise_quantize_dequantize_abs_max(input, self._quant_bits, self._quant_axis,
                                                                      self._round_type)
        if not _is_meta(scale):
            with torch.no_grad():
                self._scale._t.copy_(scale._t.reshape(self._scale._t.shape))
        return out


class MovingAverageAbsMaxScale(_ScaleHolder):
    """records the moving-average abs-max scale of its input (the layer output it observes)"""

    def __init__(self, name=None, moving_rate=0.9, dtype="float32"):
        super().__init__()
        self._moving_rate = moving_rate
        prefix = f"{name}.outscale" if name else "outscale"
        self._scale = self._state_param(prefix + ".scale", [1], 0.0)
        self._state = self._state_param(prefix + ".state", [1], 0.0)
        self._accum = self._state_param(prefix + ".accum", [1], 0.0)

    def forward(self, input):
        return QO.moving_average_abs_max_scale(input, self._scale, self._state, self._accum, self._moving_rate,
                                               not self.training)


def _get_fake_quant_type(quant_type, **kwargs):
    call_args = {"name": kwargs.get("name"), "quant_bits": kwargs.get("quant_bits", 8),
                 "dtype": kwargs.get("dtype", "float32")}
    if quant_type == "abs_max":
        call_args["quant_on_weight"] = kwargs.get("quant_on_weight", False)
    elif quant_type == "moving_average_abs_max":
        call_args["moving_rate"] = kwargs.get("moving_rate", 0.9)
    elif quant_type == "channel_wise_abs_max":
        call_args["quant_on_weight"] = kwargs.get("quant_on_weight", False)
        call_args["channel_num"] = kwargs.get("channel_num")
        call_args["quant_axis"] = kwargs.get("quant_axis", 0)
        assert call_args["channel_num"] is not None, \
            "You need to input channel_num when you use channel_wise_abs_max strategy."
    table = {"abs_max": FakeQuantAbsMax, "moving_average_abs_max": FakeQuantMovingAverageAbsMax,
             "channel_wise_abs_max": FakeQuantChannelWiseAbsMax}
    if quant_type not in table:
        raise ValueError(f"unknown fake quant type {quant_type!r}")
    return table[quant_type](**call_args)


class _QuantizedWrapper(Layer):
    """shared body of the Quantized* layers: activation + weight fake quant around the float op"""
    _weight_axis = 0

    def _setup(self, layer, weight_bits, activation_bits, moving_rate, weight_quantize_type, activation_quantize_type,
               weight_pre_layer, act_pre_layer, weight_quant_layer, act_quant_layer):
        self.weight = getattr(layer, "weight")
        self.bias = getattr(layer, "bias")
        if weight_quant_layer is not None:
            self._fake_quant_weight = weight_quant_layer()
        else:
            self._fake_quant_weight = _get_fake_quant_type(
                weight_quantize_type, name=self.weight.name, moving_rate=moving_rate, quant_bits=weight_bits,
                dtype=self._dtype, quant_on_weight=True, channel_num=self.weight.shape[self._weight_axis],
                quant_axis=self._weight_axis)
        if act_quant_layer is not None:
            self._fake_quant_input = act_quant_layer()
        else:
            self._fake_quant_input = _get_fake_quant_type(
                activation_quantize_type, name=layer.full_name(), moving_rate=moving_rate,
                quant_bits=activation_bits, dtype=self._dtype, quant_on_weight=False)
        self._act_preprocess = act_pre_layer() if act_pre_layer is not None else None
        self._weight_preprocess = weight_pre_layer() if weight_pre_layer is not None else None

    def _quant_inputs(self, input):
        if self._act_preprocess is not None:
            input = self._act_preprocess(input)
        qx = self._fake_quant_input(input)
        w = self.weight if self._weight_preprocess is None else self._weight_preprocess(self.weight)
        return qx, self._fake_quant_weight(w)


class QuantizedConv2D(_QuantizedWrapper):
    """Conv2D with fake-quantized input and weight (weight channel axis 0)"""
    _weight_axis = 0

    def __init__(self, layer, weight_bits=8, activation_bits=8, moving_rate=0.9, weight_quantize_type="abs_max",
                 activation_quantize_type="abs_max", weight_pre_layer=None, act_pre_layer=None,
                 weight_quant_layer=None, act_quant_layer=None):
        super().__init__()
        self._groups = layer._groups
        self._stride, self._padding, self._dilation = layer._stride, layer._padding, layer._dilation
        self._padding_mode = layer._padding_mode
        self._data_format = layer._data_format
        self._float_layer = [layer]   # its padding helper (not a sublayer: no duplicate parameters)
        self._setup(layer, weight_bits, activation_bits, moving_rate, weight_quantize_type, activation_quantize_type,
                    weight_pre_layer, act_pre_layer, weight_quant_layer, act_quant_layer)

    def forward(self, input):
        qx, qw = self._quant_inputs(input)
        qx, pad = self._float_layer[0]._pad_input(qx)
        return F.conv2d(qx, qw, self.bias, self._stride, pad, self._dilation, self._groups, self._data_format)


class QuantizedConv2DTranspose(_QuantizedWrapper):
    """Conv2DTranspose with fake-quantized input and weight (weight [C_in, C_out/g, kh, kw]: the
    reference quantizes along axis 0 as well)"""
    _weight_axis = 0

    def __init__(self, layer, weight_bits=8, activation_bits=8, moving_rate=0.9, weight_quantize_type="abs_max",
                 activation_quantize_type="abs_max", weight_pre_layer=None, act_pre_layer=None,
                 weight_quant_layer=None, act_quant_layer=None):
        super().__init__()
        self._groups = layer._groups
        self._stride, self._padding, self._dilation = layer._stride, layer._padding, layer._dilation
        self._output_padding = layer._output_padding
        self._data_format = layer._data_format
        self._setup(layer, weight_bits, activation_bits, moving_rate, weight_quantize_type, activation_quantize_type,
                    weight_pre_layer, act_pre_layer, weight_quant_layer, act_quant_layer)

    def forward(self, input, output_size=None):
        qx, qw = self._quant_inputs(input)
        return F.conv2d_transpose(qx, qw, self.bias, self._stride, self._padding, self._output_padding,
                                  self._dilation, self._groups, output_size, self._data_format)


class QuantizedLinear(_QuantizedWrapper):
    """Linear with fake-quantized input and weight ([in, out]: channel axis 1)"""
    _weight_axis = 1

    def __init__(self, layer, weight_bits=8, activation_bits=8, moving_rate=0.9, weight_quantize_type="abs_max",
                 activation_quantize_type="abs_max", weight_pre_layer=None, act_pre_layer=None,
                 weight_quant_layer=None, act_quant_layer=None):
        super().__init__()
        self.name = getattr(layer, "name", None)
        self._setup(layer, weight_bits, activation_bits, moving_rate, weight_quantize_type, activation_quantize_type,
                    weight_pre_layer, act_pre_layer, weight_quant_layer, act_quant_layer)

    def forward(self, input):
        qx, qw = self._quant_inputs(input)
        return F.linear(qx, qw, self.bias)


class MAOutputScaleLayer(Layer):
    """a MovingAverageAbsMaxScale observer behind ``layer``'s (single) output"""

    def __init__(self, layer=None, moving_rate=0.9, name=None, dtype="float32"):
        super().__init__()
        self._layer = layer
        self._ma_output_scale = MovingAverageAbsMaxScale(name or layer.full_name(), moving_rate, dtype)

    def forward(self, *inputs, **kwargs):
        out = self._layer(*inputs, **kwargs)
        if isinstance(out, (list, tuple, dict)):
            return out
        return self._ma_output_scale(out)


class FakeQuantMAOutputScaleLayer(Layer):
    """a moving-average fake quant-dequant of ``layer``'s output"""

    def __init__(self, layer, weight_bits=8, activation_bits=8, moving_rate=0.9, name=None, *args, **kwargs):
        super().__init__()
        self._layer = layer
        self._fake_quant_output = _get_fake_quant_type(
            "moving_average_abs_max", name=layer.full_name() if name is None else name, moving_rate=moving_rate,
            quant_bits=activation_bits, dtype=self._dtype, quant_on_weight=False)

    def forward(self, *inputs, **kwargs):
        out = self._layer(*inputs, **kwargs)
        if isinstance(out, (list, tuple)) and len(out) > 1:
            return out
        return self._fake_quant_output(out)


class QuantStub(Layer):
    """identity that marks where ImperativeQuantAware / ImperativePTQ quantize a model input"""

    def __init__(self, *args, **kwargs):
        super().__init__()

    def forward(self, input):
        return input
