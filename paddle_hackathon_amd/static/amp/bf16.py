"""``paddle.static.amp.bf16`` (reference: python/paddle/fluid/contrib/mixed_precision/bf16): the
bfloat16 variant of the static AMP rewrite (no loss scaling: bf16 has fp32's exponent range)."""
from __future__ import annotations

import contextlib

import numpy as np
import torch

from . import _StaticAMP, _cast, cast_parameters_to_fp16, fp16_guard
from ...fluid.contrib.mixed_precision import AutoMixedPrecisionLists

__all__ = ["AutoMixedPrecisionListsBF16", "bf16_guard", "decorate_bf16", "cast_model_to_bf16",
           "cast_parameters_to_bf16", "rewrite_program_bf16", "convert_float_to_uint16"]

AutoMixedPrecisionListsBF16 = AutoMixedPrecisionLists


@contextlib.contextmanager
def bf16_guard():
    with fp16_guard():
        yield


def decorate_bf16(optimizer, amp_lists=None, use_pure_bf16=False, use_bf16_guard=None):
    return _StaticAMP(optimizer, amp_lists or AutoMixedPrecisionListsBF16(), 1.0, False, 1000, 2, 1.0, 1.0, True,
                      dtype=torch.bfloat16, use_fp16_guard=bool(use_bf16_guard) if use_bf16_guard is not None
                      else use_pure_bf16, pure=use_pure_bf16)


def rewrite_program_bf16(main_prog, amp_lists=None):
    return _cast(main_prog, torch.bfloat16, amp_lists)


def cast_model_to_bf16(program, amp_lists=None, use_bf16_guard=True):
    return _cast(program, torch.bfloat16, amp_lists, use_bf16_guard, everything=True)


def cast_parameters_to_bf16(place=None, program=None, scope=None, to_bf16_var_names=None):
    return cast_parameters_to_fp16(place, program, scope, to_bf16_var_names, dtype=torch.bfloat16)


def convert_float_to_uint16(data, data_format="NCHW"):
    """fp32 numpy -> the bf16 bit patterns as uint16 (round to nearest even)"""
    t = torch.from_numpy(np.ascontiguousarray(data, dtype=np.float32)).to(torch.bfloat16)
    return t.view(torch.int16).numpy().view(np.uint16)
