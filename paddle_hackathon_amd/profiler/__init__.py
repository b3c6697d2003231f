"""``paddle.profiler`` (reference: python/paddle/profiler/{profiler,utils,profiler_statistic,
timer}.py and the C++ host tracer in paddle/fluid/platform/profiler/).

Host side: op / layer / user ranges are recorded by the native tracer in
``csrc/runtime/tracer.cpp`` (per-thread buffers, chrome-trace export). Device side: HIP
kernel and memcpy activity comes from roctracer through ``torch.profiler`` (kineto) when
``ProfilerTarget.GPU`` is requested. ``export_chrome_tracing`` merges both timelines into
one JSON file; ``summary()`` prints per-op host statistics and per-kernel device statistics.
For production kernel-level counters on MI355X use ``rocprofv3`` (see profiles/README.md).
"""
from __future__ import annotations

import contextlib
import enum
import json
import os
import socket
import tempfile
import time

from ..framework import core as _core
from ..utils import native as _native
from .timer import benchmark  # noqa: F401

__all__ = ["ProfilerState", "ProfilerTarget", "make_scheduler", "export_chrome_tracing", "export_protobuf",
           "Profiler", "RecordEvent", "load_profiler_result", "SortedKeys"]


class ProfilerState(enum.Enum):
    CLOSED = 0
    READY = 1
    RECORD = 2
    RECORD_AND_RETURN = 3


class ProfilerTarget(enum.Enum):
    CPU = 0
    GPU = 1
    MLU = 2
    CUSTOM_DEVICE = 3


class SortedKeys(enum.Enum):
    CPUTotal = 0
    CPUAvg = 1
    CPUMax = 2
    CPUMin = 3
    GPUTotal = 4
    GPUAvg = 5
    GPUMax = 6
    GPUMin = 7


class TracerEventType(enum.Enum):
    Operator = 0
    Dataloader = 1
    ProfileStep = 2
    CudaRuntime = 3
    Kernel = 4
    Memcpy = 5
    Memset = 6
    UserDefined = 7
    OperatorInner = 8
    Forward = 9
    Backward = 10
    Optimization = 11
    Communication = 12
    PythonOp = 13
    PythonUserDefined = 14


_TYPE_NAME = {TracerEventType.Operator: "Operator", TracerEventType.Dataloader: "Dataloader",
              TracerEventType.ProfileStep: "ProfileStep", TracerEventType.Forward: "Forward",
              TracerEventType.Backward: "Backward", TracerEventType.Optimization: "Optimization",
              TracerEventType.Communication: "Communication", TracerEventType.PythonOp: "PythonOp"}


@contextlib.contextmanager
def _op_range(name, type_name):
    """Used by the op dispatcher / Layer.__call__ while tracing is on."""
    tr = _native.host_tracer()
    tr.push(name, type_name)
    rf = None
    if _active is not None and _active._torch_prof is not None:
        import torch
        rf = torch.autograd.profiler.record_function(name)
        rf.__enter__()
    try:
        yield
    finally:
        if rf is not None:
            rf.__exit__(None, None, None)
        tr.pop()


class RecordEvent:
    """User range: ``with RecordEvent("fwd"):``, ``begin()/end()`` or as a decorator."""

    def __init__(self, name, event_type=TracerEventType.PythonUserDefined):
        self.name = name
        self.event_type = event_type
        self._open = False
        self._rf = None

    def begin(self):
        tr = _native.host_tracer()
        if not tr.enabled:
            return
        tr.push(self.name, _TYPE_NAME.get(self.event_type, "UserDefined"))
        if _active is not None and _active._torch_prof is not None:
            import torch
            self._rf = torch.autograd.profiler.record_function(self.name)
            self._rf.__enter__()
        self._open = True

    def end(self):
        if not self._open:
            return
        if self._rf is not None:
            self._rf.__exit__(None, None, None)
            self._rf = None
        _native.host_tracer().pop()
        self._open = False

    def __enter__(self):
        self.begin()
        return self

    def __exit__(self, *exc):
        self.end()

    def __call__(self, fn):
        import functools

        @functools.wraps(fn)
        def wrapper(*a, **k):
            with RecordEvent(self.name, self.event_type):
                return fn(*a, **k)
        return wrapper


def make_scheduler(*, closed, ready, record, repeat=0, skip_first=0):
    """step -> ProfilerState, cycling closed → ready → record (last record step returns)."""
    def sched(step):
        if step < skip_first:
            return ProfilerState.CLOSED
        step -= skip_first
        period = closed + ready + record
        if repeat > 0 and step // period >= repeat:
            return ProfilerState.CLOSED
        m = step % period
        if m < closed:
            return ProfilerState.CLOSED
        if m < closed + ready:
            return ProfilerState.READY
        return ProfilerState.RECORD if m < period - 1 else ProfilerState.RECORD_AND_RETURN
    return sched


def _default_scheduler(step):
    return ProfilerState.RECORD


def _worker_name(worker_name):
    return worker_name or f"host_{socket.gethostname()}pid_{os.getpid()}"


def export_chrome_tracing(dir_name, worker_name=None):
    def handle(prof):
        os.makedirs(dir_name, exist_ok=True)
        path = os.path.join(dir_name, f"{_worker_name(worker_name)}_time_{time.strftime('%Y_%m_%d_%H_%M_%S')}"
                                      f".paddle_trace.json")
        prof.export(path, "json")
    return handle


def export_protobuf(dir_name, worker_name=None):
    def handle(prof):
        os.makedirs(dir_name, exist_ok=True)
        path = os.path.join(dir_name, f"{_worker_name(worker_name)}_time_{time.strftime('%Y_%m_%d_%H_%M_%S')}"
                                      f".paddle_trace.pb")
        prof.export(path, "pb")
    return handle


class ProfilerResult:
    """Loaded trace: ``events`` is the list of chrome-trace event dicts."""

    def __init__(self, events):
        self.events = events

    def get_data(self):
        return self.events

    def save(self, path, format="json"):
        _write(self.events, path, format)


def _write(events, path, format):
    if format == "json":
        with open(path, "w") as f:
            json.dump({"traceEvents": events, "displayTimeUnit": "ms"}, f)
        return
    from google.protobuf import struct_pb2
    msg = struct_pb2.Struct()
    msg.update({"traceEvents": events})
    with open(path, "wb") as f:
        f.write(msg.SerializeToString())


def load_profiler_result(filename):
    if filename.endswith(".json"):
        with open(filename) as f:
            return ProfilerResult(json.load(f)["traceEvents"])
    from google.protobuf import struct_pb2, json_format
    msg = struct_pb2.Struct()
    with open(filename, "rb") as f:
        msg.ParseFromString(f.read())
    return ProfilerResult(json_format.MessageToDict(msg)["traceEvents"])


_active = None


class Profiler:
    def __init__(self, *, targets=None, scheduler=None, on_trace_ready=None, record_shapes=False,
                 profile_memory=False, timer_only=False, emit_nvtx=False, custom_device_types=None,
                 with_flops=False):
        import torch
        if targets is None:
            targets = [ProfilerTarget.CPU] + ([ProfilerTarget.GPU] if torch.cuda.is_available() else [])
        self.targets = set(targets)
        if isinstance(scheduler, (tuple, list)):
            start, end = scheduler
            scheduler = make_scheduler(closed=max(start - 1, 0), ready=1 if start > 0 else 0, record=end - start,
                                       repeat=1)
        self.scheduler = scheduler or _default_scheduler
        self.on_trace_ready = on_trace_ready or export_chrome_tracing("./profiler_log/")
        self.record_shapes, self.profile_memory, self.timer_only = record_shapes, profile_memory, timer_only
        self.step_num = 0
        self.previous_state = ProfilerState.CLOSED
        self.current_state = self.scheduler(self.step_num)
        self._torch_prof = None
        self._events = []
        self._device_events = []
        self._step_event = None
        self._timer = benchmark()

    # -- lifecycle ---------------------------------------------------------------------
    def start(self):
        global _active
        _active = self
        self._timer.begin()
        if self.timer_only:
            return
        if self.current_state in (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN):
            self._start_record()
        self._step_begin()

    def stop(self):
        global _active
        self._timer.end()
        if self.timer_only:
            _active = None
            return
        self._step_end()
        if self.current_state in (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN):
            self._stop_record()
            if self.on_trace_ready:
                self.on_trace_ready(self)
        _active = None

    def step(self, num_samples=None):
        self._timer.step(num_samples)
        if self.timer_only:
            return
        self._step_end()
        self.previous_state = self.current_state
        self.step_num += 1
        self.current_state = self.scheduler(self.step_num)
        recording = (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN)
        if self.previous_state in recording and (self.current_state not in recording
                                                 or self.previous_state == ProfilerState.RECORD_AND_RETURN):
            self._stop_record()
            if self.on_trace_ready:
                self.on_trace_ready(self)
        if self.current_state in recording and (self.previous_state not in recording
                                                or self.previous_state == ProfilerState.RECORD_AND_RETURN):
            self._start_record()
        self._step_begin()

    def step_info(self, unit=None):
        return self._timer.step_info(unit)

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *exc):
        self.stop()

    # -- recording -----------------------------------------------------------------------
    def _step_begin(self):
        if self.current_state in (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN):
            self._step_event = RecordEvent(f"ProfileStep#{self.step_num}", TracerEventType.ProfileStep)
            self._step_event.begin()

    def _step_end(self):
        if self._step_event is not None:
            self._step_event.end()
            self._step_event = None

    def _start_record(self):
        tr = _native.host_tracer()
        tr.clear()
        tr.enable(True)
        _core._mode.trace = True
        if ProfilerTarget.GPU in self.targets:
            import torch
            if torch.cuda.is_available():
                acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
                self._torch_prof = torch.profiler.profile(activities=acts, record_shapes=self.record_shapes,
                                                          profile_memory=self.profile_memory)
                self._torch_prof.__enter__()

    def _stop_record(self):
        tr = _native.host_tracer()
        _core._mode.trace = False
        with tempfile.TemporaryDirectory() as d:
            hp = os.path.join(d, "host.json")
            tr.export_chrome(hp)
            with open(hp) as f:
                self._events = json.load(f)["traceEvents"]
            self._device_events = []
            if self._torch_prof is not None:
                import torch
                torch.cuda.synchronize()
                self._torch_prof.__exit__(None, None, None)
                dp = os.path.join(d, "device.json")
                self._torch_prof.export_chrome_trace(dp)
                with open(dp) as f:
                    dev = json.load(f).get("traceEvents", [])
                self._device_events = [e for e in dev if e.get("cat") in ("kernel", "gpu_memcpy", "gpu_memset",
                                                                             "cuda_runtime", "gpu_user_annotation")]
                self._torch_prof = None
        tr.enable(False)
        tr.clear()

    # -- output ----------------------------------------------------------------------------
    def export(self, path="", format="json"):
        _write(self._events + self._device_events, path, format)

    def _stats(self):
        host, dev = {}, {}
        for e in self._events:
            if e.get("cat") == "ProfileStep":
                continue
            host.setdefault((e.get("cat"), e["name"]), []).append(e["dur"])
        for e in self._device_events:
            if e.get("cat") == "kernel":
                dev.setdefault(e["name"], []).append(e.get("dur", 0.0))
        return host, dev

    def summary(self, sorted_by=SortedKeys.CPUTotal, op_detail=True, thread_sep=False, time_unit="ms"):
        scale = {"s": 1e-6, "ms": 1e-3, "us": 1.0, "ns": 1e3}[time_unit]
        host, dev = self._stats()
        key = {SortedKeys.CPUTotal: sum, SortedKeys.CPUAvg: lambda v: sum(v) / len(v), SortedKeys.CPUMax: max,
               SortedKeys.CPUMin: min}.get(sorted_by, sum)
        lines = [f"{'Name':<48}{'Type':<14}{'Calls':>8}{'Total(' + time_unit + ')':>14}{'Avg':>12}{'Max':>12}{'Min':>12}"]
        for (cat, name), v in sorted(host.items(), key=lambda kv: -key(kv[1])):
            lines.append(f"{name[:47]:<48}{cat:<14}{len(v):>8}{sum(v) * scale:>14.4f}{sum(v) / len(v) * scale:>12.4f}"
                         f"{max(v) * scale:>12.4f}{min(v) * scale:>12.4f}")
        if dev:
            dkey = {SortedKeys.GPUAvg: lambda v: sum(v) / len(v), SortedKeys.GPUMax: max, SortedKeys.GPUMin: min}.get(
                sorted_by, sum)
            lines.append("")
            lines.append(f"{'Kernel':<62}{'Calls':>8}{'Total(' + time_unit + ')':>14}{'Avg':>12}{'Ratio(%)':>10}")
            tot = sum(sum(v) for v in dev.values()) or 1.0
            for name, v in sorted(dev.items(), key=lambda kv: -dkey(kv[1])):
                lines.append(f"{name[:61]:<62}{len(v):>8}{sum(v) * scale:>14.4f}{sum(v) / len(v) * scale:>12.4f}"
                             f"{100 * sum(v) / tot:>10.2f}")
        text = "\n".join(lines)
        print(text)
        return text
