"""``QuantizeTranspiler`` (reference python/paddle/fluid/contrib/quantize/quantize_transpiler.py:80):
the 1.x quantization-aware-training rewrite of a Program, over the slim passes of
fluid/contrib/slim/quantization (the HIP fake-quant kernels of csrc/kernels/quant.hip):

* ``training_transpile(program)`` — a fake quant-dequant op in front of every quantizable op's
  activation and weight inputs (conv2d / depthwise_conv2d / mul / fc / matmul); gradients pass
  straight through them (STE);
* ``freeze_program(program, place)`` — weights quantized in place with their scales, activation
  fake quant-dequant kept for inference;
* ``convert_to_int8(program, place)`` — int8 weight storage with a dequantize in front of the op.
"""
from __future__ import annotations

__all__ = ["QuantizeTranspiler"]

_TYPES = ("abs_max", "range_abs_max", "moving_average_abs_max")


class QuantizeTranspiler:
    def __init__(self, weight_bits=8, activation_bits=8, activation_quantize_type="abs_max",
                 weight_quantize_type="abs_max", window_size=10000, moving_rate=0.9):
        if weight_quantize_type not in _TYPES:
            raise ValueError(f"Unknown weight_quantize_type: '{weight_quantize_type}'. It can only be "
                             "'abs_max' or 'range_abs_max' or 'moving_average_abs_max'.")
        if activation_quantize_type not in _TYPES:
            raise ValueError(f"Unknown activation_quantize_type : '{activation_quantize_type}'. It can only be "
                             "'abs_max' or 'range_abs_max' or 'moving_average_abs_max'.")
        self.weight_bits, self.activation_bits = weight_bits, activation_bits
        self.weight_quantize_type = weight_quantize_type
        self.activation_quantize_type = activation_quantize_type
        self.window_size, self.moving_rate = window_size, moving_rate
        self.quantizable_op_type = ["conv2d", "depthwise_conv2d", "mul", "fc", "matmul", "matmul_v2"]

    def _graph(self, program, for_test):
        from ..slim.quantization.quantization_pass import IrGraph
        from ...framework import default_main_program
        return IrGraph(program if program is not None else default_main_program(), for_test=for_test)

    def training_transpile(self, program=None, startup_program=None):
        from ..slim.quantization.quantization_pass import QuantizationTransformPass
        g = self._graph(program, False)
        # weights take abs_max (range_abs_max is an activation scheme; the reference warns likewise)
        wq = "abs_max" if self.weight_quantize_type == "range_abs_max" else self.weight_quantize_type
        QuantizationTransformPass(weight_bits=self.weight_bits, activation_bits=self.activation_bits,
                                  activation_quantize_type=self.activation_quantize_type, weight_quantize_type=wq,
                                  window_size=self.window_size, moving_rate=self.moving_rate,
                                  quantizable_op_type=self.quantizable_op_type).apply(g)
        return g.to_program()

    def freeze_program(self, program, place, scope=None):
        from ..slim.quantization.quantization_pass import QuantizationFreezePass
        g = self._graph(program, True)
        QuantizationFreezePass(scope=scope, place=place, weight_bits=self.weight_bits,
                               activation_bits=self.activation_bits,
                               weight_quantize_type=self.weight_quantize_type).apply(g)
        return g.to_program()

    def convert_to_int8(self, program, place, scope=None):
        from ..slim.quantization.quantization_pass import ConvertToInt8Pass
        ConvertToInt8Pass(scope=scope, place=place, quantizable_op_type=self.quantizable_op_type,
                          weight_bits=self.weight_bits).apply(program)
        return program
