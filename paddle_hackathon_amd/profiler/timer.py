"""Throughput timer behind ``Profiler.step_info`` / ``timer_only`` mode (reference:
python/paddle/profiler/timer.py): reader_cost, batch_cost and ips over the last steps."""
from __future__ import annotations

import time


class _Stat:
    def __init__(self):
        self.reset()

    def reset(self):
        self.total, self.count, self.last = 0.0, 0, 0.0

    def add(self, v):
        self.total += v
        self.count += 1
        self.last = v

    @property
    def avg(self):
        return self.total / self.count if self.count else 0.0


class Benchmark:
    def __init__(self):
        self.reader = _Stat()
        self.batch = _Stat()
        self.samples = 0
        self.unit = "samples"
        self._t0 = self._tr = None
        self.running = False

    def begin(self):
        self.running = True
        self._t0 = self._tr = time.perf_counter()

    def before_reader(self):
        self._tr = time.perf_counter()

    def after_reader(self):
        if self._tr is not None:
            self.reader.add(time.perf_counter() - self._tr)

    def step(self, num_samples=None):
        if not self.running:
            return
        now = time.perf_counter()
        self.batch.add(now - self._t0)
        self._t0 = now
        if num_samples is not None:
            self.samples += num_samples

    def end(self):
        self.running = False

    def step_info(self, unit=None):
        unit = unit or self.unit
        msg = f"reader_cost: {self.reader.avg:.5f} s batch_cost: {self.batch.avg:.5f} s"
        if self.samples and self.batch.total > 0:
            msg += f" ips: {self.samples / self.batch.total:.3f} {unit}/s"
        self.reader.reset()
        self.batch.reset()
        self.samples = 0
        return msg


def benchmark():
    return Benchmark()
