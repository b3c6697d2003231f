"""Layers PTQ can calibrate (reference: imperative/ptq_registry.py)."""
from __future__ import annotations

__all__ = ["PTQRegistry"]


class LayerInfo:
    """argnames of a layer's inputs, weights and outputs"""

    def __init__(self, layer, input_names, weight_names, output_names):
        self.layer, self.input_names, self.weight_names, self.output_names = layer, input_names, weight_names, \
            output_names


def _infos():
    from ...... import nn
    L = [LayerInfo(nn.Conv2D, ["Input"], ["Filter"], ["Output"]),
         LayerInfo(nn.Linear, ["X"], ["Y"], ["Out"]),
         LayerInfo(nn.BatchNorm2D, ["X"], [], ["Y"]),
         LayerInfo(nn.AdaptiveMaxPool2D, ["X"], [], ["Out"]),
         LayerInfo(nn.AdaptiveAvgPool2D, ["X"], [], ["Out"]),
         LayerInfo(nn.AvgPool2D, ["X"], [], ["Out"]),
         LayerInfo(nn.MaxPool2D, ["X"], [], ["Out"]),
         LayerInfo(nn.ReLU, ["X"], [], ["Out"]),
         LayerInfo(nn.ReLU6, ["X"], [], ["Out"]),
         LayerInfo(nn.Hardswish, ["X"], [], ["Out"]),
         LayerInfo(nn.Swish, ["X"], [], ["Out"]),
         LayerInfo(nn.Sigmoid, ["X"], [], ["Out"]),
         LayerInfo(nn.Softmax, ["X"], [], ["Out"]),
         LayerInfo(nn.Tanh, ["X"], [], ["Out"]),
         LayerInfo(nn.quant.add, ["X", "Y"], [], ["Out"])]
    return L


class PTQRegistry:
    supported_layers_map = {}
    registered_layers_map = {}
    is_inited = False

    @classmethod
    def _init(cls):
        if not cls.is_inited:
            for info in _infos():
                cls.supported_layers_map[info.layer] = info
            from ...... import nn
            cls.registered_layers_map = {k: v for k, v in cls.supported_layers_map.items()
                                         if k in (nn.Conv2D, nn.Linear)}
            cls.is_inited = True

    @classmethod
    def _cls(cls, layer):
        return layer if isinstance(layer, type) else type(layer)

    @classmethod
    def is_supported_layer(cls, layer):
        cls._init()
        return cls._cls(layer) in cls.supported_layers_map

    @classmethod
    def is_registered_layer(cls, layer):
        cls._init()
        return cls._cls(layer) in cls.registered_layers_map

    @classmethod
    def is_simulated_quant_layer(cls, layer):
        from ...... import nn
        return cls._cls(layer) in (nn.Conv2D, nn.Linear)

    @classmethod
    def layer_info(cls, layer):
        cls._init()
        return cls.supported_layers_map[cls._cls(layer)]
