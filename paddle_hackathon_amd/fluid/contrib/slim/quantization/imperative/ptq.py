"""Dygraph post-training quantization (reference: fluid/contrib/slim/quantization/imperative/ptq.py:39
ImperativePTQ).

``quantize(model)`` (a copy unless ``inplace``) hooks every Conv2D / Linear: each calibration
forward feeds the layer's input to its config's activation quantizer (AbsmaxQuantizer /
HistQuantizer / KLQuantizer) and its weight to the weight quantizer. ``save_quantized_model``
computes the thresholds, swaps each calibrated layer for its Quantized* wrapper whose input
quantizer is frozen at the calibrated scale and whose weight is quantized per channel, and
exports through ImperativeQuantAware's path (reference fake-quant op types, out_threshold
attributes)."""
from __future__ import annotations

import copy

import numpy as np
import torch

from ......nn import quant as Q
from ......nn.layer.layers import Layer
from ...... import nn
from .ptq_config import default_ptq_config
from .ptq_registry import PTQRegistry
from .qat import _children, _set_child, fuse_conv_bn

__all__ = ["ImperativePTQ"]


class _FrozenActQuant(Layer):
    """quant-dequant with a calibrated per-tensor scale (recorded as a frozen fake-quant op)"""

    def __init__(self, threshold, bits=8):
        super().__init__()
        from ......framework.param_attr import ParamAttr
        from ......nn.initializer import Constant
        self._bits = bits
        self._scale = self.create_parameter([1], attr=ParamAttr(initializer=Constant(float(threshold)),
                                                                trainable=False), dtype="float32")
        self._scale.stop_gradient = True

    def forward(self, x):
        return Q.ops.fake_quantize_dequantize_fixed_scale(x, self._scale, self._bits)


class ImperativePTQ:
    def __init__(self, quant_config=default_ptq_config):
        self._quant_config = quant_config

    def quantize(self, model, inplace=False, fuse=False, fuse_list=None):
        assert isinstance(model, nn.Layer), "The model must be the instance of paddle.nn.Layer."
        if not inplace:
            model = copy.deepcopy(model)
        if fuse:
            model.eval()
            fuse_conv_bn(model)
        for name, layer in model.named_sublayers():
            if PTQRegistry.is_simulated_quant_layer(layer) and not getattr(layer, "skip_quant", False):
                cfg = copy.deepcopy(self._quant_config)
                layer._quant_config = cfg
                cfg.quant_hook_handle = layer.register_forward_post_hook(self._sample_hook)
        return model

    @staticmethod
    def _sample_hook(layer, inputs, output):
        cfg = layer._quant_config
        x = inputs[0] if isinstance(inputs, (tuple, list)) else inputs
        cfg.in_act_quantizer.sample_data(layer, [x])
        cfg.out_act_quantizer.sample_data(layer, [output])
        cfg.wt_quantizer.sample_data(layer, [layer.weight])
        cfg.enable_in_act_quantizer = True

    def _convert(self, parent):
        for name, child in _children(parent):
            cfg = getattr(child, "_quant_config", None)
            if cfg is not None and cfg.enable_in_act_quantizer:
                for q in (cfg.in_act_quantizer, cfg.out_act_quantizer, cfg.wt_quantizer):
                    q.cal_thresholds()
                if cfg.quant_hook_handle is not None:
                    cfg.quant_hook_handle.remove()
                t = float(np.asarray(cfg.in_act_quantizer.thresholds[0]).max())
                bits = cfg.in_act_quantizer.quant_bits
                wrap = {nn.Conv2D: Q.QuantizedConv2D, nn.Linear: Q.QuantizedLinear}[type(child)]
                q = wrap(child, weight_bits=cfg.wt_quantizer.quant_bits, activation_bits=bits,
                         weight_quantize_type="channel_wise_abs_max",
                         act_quant_layer=lambda t=t, bits=bits: _FrozenActQuant(t, bits))
                q._out_threshold = float(np.asarray(cfg.out_act_quantizer.thresholds[0]).max())
                _set_child(parent, name, q)
            else:
                self._convert(child)

    def save_quantized_model(self, model, path, input_spec=None, **config):
        from .qat import ImperativeQuantAware
        self._convert(model)
        ImperativeQuantAware().save_quantized_model(model, path, input_spec=input_spec, **config)
        return model
