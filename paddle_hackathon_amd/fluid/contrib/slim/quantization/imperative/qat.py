"""Dygraph quantization-aware training (reference: fluid/contrib/slim/quantization/imperative/qat.py:45
ImperativeQuantAware, with ImperativeQuantizeInputs / ImperativeQuantizeOutputs).

``quantize(model)`` rewrites the model in place: every layer of ``quantizable_layer_type``
(Conv2D, Linear, Conv2DTranspose) becomes its Quantized* wrapper (fake-quantized input and weight,
nn/quant/quant_layers.py), the float functional layers (nn.quant.add ...) get a fake-quantized
output, and the activation layers an output-scale observer. Training then runs as usual — the
fake-quant ops run on the HIP kernels with straight-through gradients.

``save_quantized_model(model, path, input_spec)`` exports the eval-mode model through jit.save:
the weights' fake quant-dequant ops and the activations' frozen (is_test) moving-average ops are
written as reference fake-quant op types; the observers' scales become ``out_threshold``
attributes of their producer ops (OutScaleForInferencePass). ``onnx_format=True`` writes
quantize_linear / dequantize_linear pairs with int8 weights instead.
"""
from __future__ import annotations

import torch

from ......nn import quant as Q
from ...... import nn
from .. import quantization_pass as QP

__all__ = ["ImperativeQuantAware"]

_LAYERS = {"Conv2D": "Conv2D", "Linear": "Linear", "Conv2DTranspose": "Conv2DTranspose"}
_WRAP = {"Conv2D": Q.QuantizedConv2D, "Linear": Q.QuantizedLinear, "Conv2DTranspose": Q.QuantizedConv2DTranspose}
_OUTPUT_OBSERVED = ("ReLU", "ReLU6", "LeakyReLU", "PReLU", "Sigmoid", "Tanh", "Softmax", "Swish", "Hardswish",
                    "AvgPool2D", "MaxPool2D", "AdaptiveAvgPool2D", "AdaptiveMaxPool2D", "BatchNorm", "BatchNorm2D",
                    "LayerNorm", "GroupNorm")


def _children(layer):
    return list(layer._sub_layers.items())


def _set_child(parent, name, child):
    parent._sub_layers[name] = child
    if name in parent.__dict__:
        parent.__dict__[name] = child


def fuse_conv_bn(model):
    """fold each BatchNorm that directly follows a Conv2D in a Sequential into the conv (eval-mode
    statistics), leaving an Identity (reference imperative/fuse_utils.py)"""
    for name, child in _children(model):
        if isinstance(child, nn.Sequential):
            items = list(child._sub_layers.items())
            for (n1, a), (n2, b) in zip(items, items[1:]):
                if isinstance(a, nn.Conv2D) and isinstance(b, (nn.BatchNorm2D, nn.BatchNorm)):
                    _fold(a, b)
                    _set_child(child, n2, nn.Identity())
        fuse_conv_bn(child)
    return model


def _fold(conv, bn):
    with torch.no_grad():
        w = conv.weight._t
        mean, var = bn._mean._t.float(), bn._variance._t.float()
        gamma = bn.weight._t.float() if bn.weight is not None else torch.ones_like(mean)
        beta = bn.bias._t.float() if bn.bias is not None else torch.zeros_like(mean)
        inv = gamma / torch.sqrt(var + bn._epsilon)
        w.copy_((w.float() * inv.reshape(-1, 1, 1, 1)).to(w.dtype))
        b0 = conv.bias._t.float() if conv.bias is not None else torch.zeros_like(mean)
        nb = (b0 - mean) * inv + beta
        if conv.bias is None:
            conv.bias = conv.create_parameter([nb.numel()], is_bias=True)
        conv.bias._t.copy_(nb.to(conv.bias._t.dtype))


class ImperativeQuantAware:
    def __init__(self, quantizable_layer_type=("Conv2D", "Linear", "Conv2DTranspose"),
                 weight_quantize_type="abs_max", activation_quantize_type="moving_average_abs_max", weight_bits=8,
                 activation_bits=8, moving_rate=0.9, fuse_conv_bn=False, weight_preprocess_layer=None,
                 act_preprocess_layer=None, weight_quantize_layer=None, act_quantize_layer=None, onnx_format=False):
        types = []
        for t in quantizable_layer_type:
            name = t if isinstance(t, str) else t.__name__
            if name not in _WRAP:
                raise ValueError(f"{name} is not a quantizable layer type (one of {sorted(_WRAP)})")
            types.append(name)
        if weight_quantize_type not in ("abs_max", "channel_wise_abs_max"):
            raise ValueError(f"unsupported weight_quantize_type {weight_quantize_type!r}")
        if activation_quantize_type not in ("abs_max", "moving_average_abs_max"):
            raise ValueError(f"unsupported activation_quantize_type {activation_quantize_type!r}")
        self._types = tuple(types)
        self._kw = dict(weight_bits=weight_bits, activation_bits=activation_bits, moving_rate=moving_rate,
                        weight_quantize_type=weight_quantize_type, activation_quantize_type=activation_quantize_type,
                        weight_pre_layer=weight_preprocess_layer, act_pre_layer=act_preprocess_layer,
                        weight_quant_layer=weight_quantize_layer, act_quant_layer=act_quantize_layer)
        self._moving_rate = moving_rate
        self._abits = activation_bits
        self._fuse = fuse_conv_bn
        self._onnx = onnx_format

    def quantize(self, model):
        assert isinstance(model, nn.Layer), "The model must be the instance of paddle.nn.Layer."
        if self._fuse:
            model.eval()
            fuse_conv_bn(model)
            model.train()
        self._rewrite(model)
        return model

    def _rewrite(self, parent):
        for name, child in _children(parent):
            cls = type(child).__name__
            if getattr(child, "skip_quant", False):
                continue
            if cls in self._types and cls in _WRAP and not isinstance(child, Q.quant_layers._QuantizedWrapper):
                _set_child(parent, name, _WRAP[cls](child, **self._kw))
            elif isinstance(child, (Q.add, Q.subtract, Q.multiply, Q.divide)):
                _set_child(parent, name, Q.FakeQuantMAOutputScaleLayer(child, activation_bits=self._abits,
                                                                       moving_rate=self._moving_rate))
            elif cls in _OUTPUT_OBSERVED:
                _set_child(parent, name, Q.MAOutputScaleLayer(child, self._moving_rate))
            else:
                self._rewrite(child)

    def save_quantized_model(self, layer, path, input_spec=None, **config):
        from ...... import jit, static
        was = layer.training
        layer.eval()
        try:
            jit.save(layer, path, input_spec=input_spec, **config)
        finally:
            if was:
                layer.train()
        prog, feeds, fetches = static.load_inference_model(path)
        QP.OutScaleForInferencePass().apply(prog)
        if self._onnx:
            QP.ReplaceFakeQuantDequantPass().apply(prog)
            QP.QuantWeightPass().apply(prog)
        blk = prog.global_block()
        static.save_inference_model(path, [blk.vars[n] for n in feeds], list(fetches), program=prog)
