"""``paddle.fluid.reader`` (reference: python/paddle/fluid/reader.py): ``DataLoader`` (2.x
dataset loader plus the 1.x ``from_generator`` / ``from_dataset`` constructors) and ``PyReader``."""
from __future__ import annotations

from ..io import DataLoader as _DL, default_collate_fn  # noqa: F401
from .layers.io import PyReader as _PyReader

__all__ = ["PyReader", "DataLoader", "default_collate_fn"]


class _GeneratorLoader(_PyReader):
    """iterable loader over feed variables (``DataLoader.from_generator``)"""

    def __init__(self, feed_list=None, capacity=64, iterable=True, return_list=False, drop_last=True):
        super().__init__(feed_list or [], capacity, iterable, return_list)
        self.drop_last = drop_last

    def set_sample_generator(self, sample_generator, batch_size, drop_last=True, places=None):
        self.decorate_sample_generator(sample_generator, batch_size, drop_last, places)
        return self

    def set_sample_list_generator(self, reader, places=None):
        self.decorate_paddle_reader(reader, places)
        return self

    def set_batch_generator(self, reader, places=None):
        self.decorate_tensor_provider(reader, places)
        return self

    def __iter__(self):
        if not self.feed_vars:      # dygraph: yield the batches as tensor lists
            from ..framework.core import to_tensor
            for batch in self._source():
                yield [to_tensor(b) for b in batch]
            return
        yield from super().__iter__()


class DataLoader(_DL):
    @staticmethod
    def from_generator(feed_list=None, capacity=None, use_double_buffer=True, iterable=True, return_list=False,
                       use_multiprocess=False, drop_last=True):
        return _GeneratorLoader(feed_list, capacity or 64, iterable, return_list, drop_last)

    @staticmethod
    def from_dataset(dataset, places, drop_last=True):
        return _DL(dataset, batch_size=1, drop_last=drop_last)


class PyReader(_GeneratorLoader):
    def __init__(self, feed_list=None, capacity=None, use_double_buffer=True, iterable=True, return_list=False):
        super().__init__(feed_list, capacity or 64, iterable, return_list)
