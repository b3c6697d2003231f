"""``paddle.device.cuda`` — HIP streams/events/memory stats for the MI355X (reference:
python/paddle/device/cuda/__init__.py, streams.py). Streams are HIP streams; on MI355X use
separate streams to overlap RCCL collectives and H2D copies with compute."""
from __future__ import annotations

import contextlib

import torch

__all__ = ["Stream", "Event", "current_stream", "synchronize", "device_count", "empty_cache",
           "max_memory_allocated", "max_memory_reserved", "memory_allocated", "memory_reserved",
           "stream_guard", "get_device_properties", "get_device_name", "get_device_capability"]

from . import graphs  # noqa: E402,F401  (hipGraph capture: paddle.device.cuda.graphs)


def _dev(device):
    if device is None:
        return torch.cuda.current_device()
    if isinstance(device, int):
        return device
    if hasattr(device, "get_device_id"):
        return device.get_device_id()
    s = str(device)
    return int(s.split(":")[1]) if ":" in s else 0


class Stream:
    def __init__(self, device=None, priority=2, stream=None):
        self._s = stream if stream is not None else torch.cuda.Stream(device=_dev(device),
                                                                       priority=-1 if priority == 1 else 0)

    def wait_event(self, event):
        self._s.wait_event(event._e)

    def wait_stream(self, stream):
        self._s.wait_stream(stream._s)

    def query(self):
        return self._s.query()

    def synchronize(self):
        self._s.synchronize()

    def record_event(self, event=None):
        event = event or Event()
        event.record(self)
        return event

    @property
    def cuda_stream(self):
        return self._s.cuda_stream


class Event:
    def __init__(self, enable_timing=False, blocking=False, interprocess=False):
        self._e = torch.cuda.Event(enable_timing=enable_timing, blocking=blocking, interprocess=interprocess)

    def record(self, stream=None):
        self._e.record(stream._s if stream is not None else None)

    def query(self):
        return self._e.query()

    def synchronize(self):
        self._e.synchronize()

    def elapsed_time(self, end):
        return self._e.elapsed_time(end._e)


def current_stream(device=None):
    return Stream(stream=torch.cuda.current_stream(_dev(device)))


def synchronize(device=None):
    torch.cuda.synchronize(_dev(device) if device is not None else None)


def device_count():
    return torch.cuda.device_count()


def empty_cache():
    if torch.cuda.is_available():
        torch.cuda.empty_cache()


def max_memory_allocated(device=None):
    return torch.cuda.max_memory_allocated(_dev(device))


def max_memory_reserved(device=None):
    return torch.cuda.max_memory_reserved(_dev(device))


def memory_allocated(device=None):
    return torch.cuda.memory_allocated(_dev(device))


def memory_reserved(device=None):
    return torch.cuda.memory_reserved(_dev(device))


@contextlib.contextmanager
def stream_guard(stream):
    if stream is None:
        yield
        return
    with torch.cuda.stream(stream._s):
        yield


def get_device_properties(device=None):
    return torch.cuda.get_device_properties(_dev(device))


def get_device_name(device=None):
    return torch.cuda.get_device_name(_dev(device))


def get_device_capability(device=None):
    return torch.cuda.get_device_capability(_dev(device))
