"""Framework-level fake-quantization ops, named after the reference op types they record as
(paddle/fluid/operators/fake_quantize_op.cc, fake_dequantize_op.cc, quantize_linear_op.cc).

Each takes / returns framework Tensors, records one op in a static Program (framework/dispatch.py)
and runs the HIP kernels of csrc/kernels/quant.hip on the GPU (ops/quant.py). Moving-average
state (``scale``, ``state``, ``accum``) is updated in place, as the reference's in-place
OutScale / OutState / OutAccum outputs; the quant-dequant outputs carry the straight-through
gradient."""
from __future__ import annotations

from ...framework.core import Tensor, _wrap
from ...framework.dispatch import register_ops
from ...ops import quant as Q

__all__ = ["fake_quantize_dequantize_abs_max", "fake_quantize_abs_max",
           "fake_channel_wise_quantize_dequantize_abs_max", "fake_channel_wise_quantize_abs_max",
           "fake_quantize_dequantize_moving_average_abs_max", "fake_quantize_moving_average_abs_max",
           "moving_average_abs_max_scale", "fake_dequantize_max_abs", "fake_channel_wise_dequantize_max_abs",
           "quantize_linear", "dequantize_linear", "fake_quantize_dequantize_fixed_scale"]


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def fake_quantize_dequantize_abs_max(x, bit_length=8, round_type=1):
    """-> (Out, OutScale[1])"""
    out, s = Q.fake_quantize_dequantize_abs_max(_t(x), bit_length, round_type)
    return _wrap(out), _wrap(s)


def fake_quantize_abs_max(x, bit_length=8, round_type=1):
    out, s = Q.fake_quantize_abs_max(_t(x), bit_length, round_type)
    return _wrap(out), _wrap(s)


def fake_channel_wise_quantize_dequantize_abs_max(x, bit_length=8, quant_axis=0, round_type=1):
    out, s = Q.fake_channel_wise_quantize_dequantize_abs_max(_t(x), bit_length, quant_axis, round_type)
    return _wrap(out), _wrap(s)


def fake_channel_wise_quantize_abs_max(x, bit_length=8, quant_axis=0, round_type=1):
    out, s = Q.fake_channel_wise_quantize_abs_max(_t(x), bit_length, quant_axis, round_type)
    return _wrap(out), _wrap(s)


def fake_quantize_dequantize_moving_average_abs_max(x, in_scale, in_state, in_accum, bit_length=8, moving_rate=0.9,
                                                    is_test=False, round_type=1):
    return _wrap(Q.fake_quantize_dequantize_moving_average_abs_max(
        _t(x), _t(in_scale), _t(in_state), _t(in_accum), bit_length, moving_rate, is_test, round_type))


def fake_quantize_moving_average_abs_max(x, in_scale, in_state, in_accum, bit_length=8, moving_rate=0.9,
                                         is_test=False, round_type=1):
    return _wrap(Q.fake_quantize_moving_average_abs_max(
        _t(x), _t(in_scale), _t(in_state), _t(in_accum), bit_length, moving_rate, is_test, round_type))


def moving_average_abs_max_scale(x, in_scale, in_state, in_accum, moving_rate=0.9, is_test=False):
    return _wrap(Q.moving_average_abs_max_scale(_t(x), _t(in_scale), _t(in_state), _t(in_accum), moving_rate,
                                                is_test))


def fake_quantize_dequantize_fixed_scale(x, scale, bit_length=8, round_type=1, quant_axis=None):
    """quant-dequant with a calibrated (frozen) scale: the inference form of the activation
    fake-quant ops (is_test=True) and of PTQ's inserted quant-dequant pairs"""
    xt = _t(x)
    return _wrap(Q.ste(xt, Q.quant_dequant(xt, _t(scale), bit_length, round_type, quant_axis=quant_axis)))


def fake_dequantize_max_abs(x, scale, max_range=127.0):
    return _wrap(Q.fake_dequantize_max_abs(_t(x), _t(scale), max_range))


def fake_channel_wise_dequantize_max_abs(x, scales, quant_bits=(8,), quant_axis=0):
    return _wrap(Q.fake_channel_wise_dequantize_max_abs(_t(x), _t(scales), quant_bits, quant_axis))


def quantize_linear(x, scale, zero_point=None, bit_length=8, quant_axis=-1, round_type=0):
    return _wrap(Q.quantize_linear(_t(x), _t(scale), _t(zero_point), bit_length, quant_axis, round_type))


def dequantize_linear(x, scale, zero_point=None, bit_length=8, quant_axis=-1):
    return _wrap(Q.dequantize_linear(_t(x), _t(scale), _t(zero_point), bit_length, quant_axis))


register_ops(globals(), __all__)
