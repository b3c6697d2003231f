"""``DataFeeder`` (reference: python/paddle/fluid/data_feeder.py): turns minibatches of per-sample
tuples into a feed dict, LoD tensors for lod_level > 0 variables."""
from __future__ import annotations

import numpy as np

from .framework import default_main_program
from .lod_tensor import create_lod_tensor
from ..framework.core import convert_dtype as _convert_dtype

__all__ = ["DataFeeder", "convert_dtype", "check_type", "check_dtype", "check_variable_and_dtype"]


def convert_dtype(dtype):
    import torch
    d = _convert_dtype(dtype)
    return {torch.float32: "float32", torch.float64: "float64", torch.float16: "float16", torch.bfloat16: "uint16",
            torch.int32: "int32", torch.int64: "int64", torch.bool: "bool", torch.uint8: "uint8",
            torch.int8: "int8", torch.int16: "int16"}.get(d, str(d))


def check_type(input, input_name, expected_type, op_name, extra_message=""):
    if not isinstance(input, expected_type):
        raise TypeError(f"The type of '{input_name}' in {op_name} must be {expected_type}, but received "
                        f"{type(input)}. {extra_message}")


def check_dtype(input_dtype, input_name, expected_dtype, op_name, extra_message=""):
    if convert_dtype(input_dtype) not in (expected_dtype if isinstance(expected_dtype, (list, tuple))
                                          else [expected_dtype]):
        raise TypeError(f"The data type of '{input_name}' in {op_name} must be {expected_dtype}, but received "
                        f"{convert_dtype(input_dtype)}. {extra_message}")


def check_variable_and_dtype(input, input_name, expected_dtype, op_name, extra_message=""):
    check_dtype(input.dtype, input_name, expected_dtype, op_name, extra_message)


class DataFeeder:
    def __init__(self, feed_list, place, program=None):
        prog = program or default_main_program()
        self.vars = [prog.global_block().var(v) if isinstance(v, str) else v for v in feed_list]
        self.place = place

    def feed(self, iterable):
        cols = [[] for _ in self.vars]
        for sample in iterable:
            if len(sample) != len(self.vars):
                raise ValueError(f"sample has {len(sample)} fields, feed_list has {len(self.vars)}")
            for c, v in zip(cols, sample):
                c.append(v)
        out = {}
        for v, col in zip(self.vars, cols):
            lod_level = getattr(v, "lod_level", 0) or 0
            dt = convert_dtype(v.dtype)
            if lod_level > 0:
                lens = [len(s) for s in col]
                arr = np.concatenate([np.asarray(s, dtype=dt).reshape(len(s), -1) for s in col])
                out[v.name] = create_lod_tensor(arr, [lens], self.place)
            else:
                arr = np.asarray(col, dtype=dt)
                shp = [s for s in (getattr(v, "declared_shape", None) or v.shape)]
                if shp and all(isinstance(s, int) for s in shp):
                    arr = arr.reshape([-1] + [s for s in shp[1:]]) if len(shp) > 1 else arr.reshape(-1)
                out[v.name] = arr
        return out

    def feed_parallel(self, iterable, num_places=None):
        for batch in iterable:
            yield self.feed(batch)

    def decorate_reader(self, reader, multi_devices=False, num_places=None, drop_last=True):
        def gen():
            for batch in reader():
                yield self.feed(batch)
        return gen
