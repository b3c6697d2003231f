"""``fluid.layers`` data / reader layers (reference: python/paddle/fluid/layers/io.py).

``data`` declares a feed Variable (prepending the batch dimension like 1.x). ``py_reader`` /
``create_py_reader_by_data`` attach a Python-fed reader to the current Program: after
``reader.start()`` every ``Executor.run`` without a feed pulls the next batch, and
``fluid.core.EOFException`` ends the pass (the executor hook is in static/program.py)."""
from __future__ import annotations

import numpy as np
import torch

from ... import static as _static
from ...static import program as P
from ._common import T, W, dev
from .. import core as fcore

__all__ = ["data", "read_file", "double_buffer", "py_reader", "create_py_reader_by_data", "load"]


def data(name, shape, append_batch_size=True, dtype="float32", lod_level=0, type=None, stop_gradient=True):
    shape = list(shape)
    for i, s in enumerate(shape):
        if s is None:
            shape[i] = -1
            append_batch_size = False
        elif s < 0:
            append_batch_size = False
    if append_batch_size:
        shape = [-1] + shape
    v = _static.data(name, shape, dtype, lod_level)
    v.stop_gradient = stop_gradient
    v.lod_level = lod_level
    return v


class PyReader:
    """queue of feed dicts pulled by Executor.run (reference fluid/reader.py PyReader)"""

    def __init__(self, feed_vars, capacity=64, iterable=False, return_list=False):
        self.feed_vars = list(feed_vars)
        self.capacity = capacity
        self.iterable, self.return_list = iterable, return_list
        self._source = None
        self._it = None
        prog = P.default_main_program()
        prog.__dict__.setdefault("_py_readers", []).append(self)

    # sources ------------------------------------------------------------------
    def decorate_paddle_reader(self, reader, places=None):
        """``reader()`` yields batches: lists of per-sample tuples"""
        def gen():
            for batch in reader():
                cols = list(zip(*batch))
                yield [np.stack([np.asarray(c) for c in col]) for col in cols]
        self._source = gen

    decorate_sample_list_generator = decorate_paddle_reader

    def decorate_tensor_provider(self, reader, places=None):
        """``reader()`` yields lists of arrays, one per feed variable"""
        self._source = lambda: (list(b) for b in reader())

    decorate_batch_generator = decorate_tensor_provider

    def decorate_sample_generator(self, sample_generator, batch_size, drop_last=True, places=None):
        def gen():
            buf = []
            for s in sample_generator():
                buf.append(s)
                if len(buf) == batch_size:
                    yield [np.stack([np.asarray(c) for c in col]) for col in zip(*buf)]
                    buf = []
            if buf and not drop_last:
                yield [np.stack([np.asarray(c) for c in col]) for col in zip(*buf)]
        self._source = gen

    set_sample_generator = decorate_sample_generator
    set_sample_list_generator = decorate_paddle_reader
    set_batch_generator = decorate_tensor_provider

    # control ------------------------------------------------------------------
    def start(self):
        if self._source is None:
            raise RuntimeError("py_reader: decorate a data source before start()")
        self._it = iter(self._source())

    def reset(self):
        self._it = None

    def _next_feed(self):
        if self._it is None:
            return None
        try:
            batch = next(self._it)
        except StopIteration:
            self._it = None
            raise fcore.EOFException("There is no next data.")
        return {v.name: b for v, b in zip(self.feed_vars, batch)}

    def __iter__(self):
        for batch in self._source():
            feed = {v.name: b for v, b in zip(self.feed_vars, batch)}
            yield [feed[v.name] for v in self.feed_vars] if self.return_list else [feed]

    def __call__(self):
        return iter(self)


def py_reader(capacity, shapes, dtypes, lod_levels=None, name=None, use_double_buffer=True):
    base = name or "py_reader"
    vs = [_static.data(f"{base}_{i}", list(s), d) for i, (s, d) in enumerate(zip(shapes, dtypes))]
    return PyReader(vs, capacity)


def create_py_reader_by_data(capacity, feed_list, name=None, use_double_buffer=True):
    return PyReader(feed_list, capacity)


def read_file(reader):
    vs = reader.feed_vars
    return vs[0] if len(vs) == 1 else vs


def double_buffer(reader, place=None, name=None):
    return reader


def load(out, file_path, load_as_fp16=None):
    """fill ``out`` from a file written by ``fluid.io.save_vars`` / ``paddle.save`` (one tensor)"""
    from ...framework.io import load as _load
    val = _load(file_path)
    t = T(val) if hasattr(val, "_t") else torch.as_tensor(np.asarray(val), device=dev())
    if load_as_fp16:
        t = t.half()
    out._t = t.to(out._t.device) if out._t.device.type != "meta" else t
    return out


_ = W
