"""``paddle.fluid.profiler`` (reference: python/paddle/fluid/profiler.py): the 1.x profiler
context managers over the framework profiler (host spans + HIP kernel timeline)."""
from __future__ import annotations

import contextlib

from .. import profiler as _p

__all__ = ["cuda_profiler", "reset_profiler", "profiler", "start_profiler", "stop_profiler"]

_state = {"prof": None}


@contextlib.contextmanager
def cuda_profiler(output_file, output_mode=None, config=None):
    """kept for source compatibility; device timelines come from ``profiler()`` / rocprofv3"""
    yield


def reset_profiler():
    _state["prof"] = None


def start_profiler(state="All", tracer_option="Default"):
    targets = [_p.ProfilerTarget.CPU] if state == "CPU" else [_p.ProfilerTarget.CPU, _p.ProfilerTarget.GPU]
    prof = _p.Profiler(targets=targets)
    prof.start()
    _state["prof"] = prof


def stop_profiler(sorted_key=None, profile_path="/tmp/profile"):
    prof = _state["prof"]
    if prof is None:
        return
    prof.stop()
    try:
        prof.export(profile_path + ".json" if not profile_path.endswith(".json") else profile_path)
    except Exception:
        pass
    prof.summary()
    _state["prof"] = None


@contextlib.contextmanager
def profiler(state="All", sorted_key=None, profile_path="/tmp/profile", tracer_option="Default"):
    start_profiler(state, tracer_option)
    try:
        yield
    finally:
        stop_profiler(sorted_key, profile_path)
