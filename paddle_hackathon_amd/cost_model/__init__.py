"""``paddle.cost_model`` (reference: python/paddle/cost_model/cost_model.py and the C++
``core.CostModel`` of paddle/fluid/framework/ir/cost_model.cc).

* ``fluid.core.CostModel().profile_measure(main, startup, device, ["time"])`` runs the startup
  program, then the main program once with a per-op timer in the static executor
  (static/program.py run_block: the device is synchronised around every op) and returns a
  :class:`CostData` with the whole-program and per-op times in milliseconds.
* :class:`CostModel` keeps the reference's Python surface: ``build_program``, ``profile_measure``
  and the static per-op benchmark table (``static_cost_data`` / ``get_static_op_time``). The
  table shipped here was measured on MI355X by ``tools/gen_static_op_benchmark.py`` (the
  reference's holds V100 numbers): ``op``, ``config``, ``paddle_gpu_time`` (forward, ms) and
  ``paddle_gpu_time_backward`` (forward + backward, ms).
"""
from __future__ import annotations

import json
import os
import time

__all__ = ["CostModel", "CostData"]

_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "static_op_benchmark_mi355x.json")


class CostData:
    """measured costs of one program run (reference: core.CostData)"""

    def __init__(self, op_times_ms=(), whole_ms=0.0, op_types=()):
        self._ops = list(op_times_ms)
        self._types = list(op_types)
        self._whole = float(whole_ms)

    def get_whole_time_ms(self):
        return self._whole

    def get_op_time_ms(self, op_id):
        return self._ops[op_id]

    def get_op_num(self):
        return len(self._ops)

    def get_op_type(self, op_id):
        return self._types[op_id]


def _sync(device):
    import torch
    if device != "cpu" and torch.cuda.is_available():
        torch.cuda.synchronize()


class _CoreCostModel:
    """``fluid.core.CostModel``"""

    def profile_measure(self, main_program, startup_program, device="gpu", fetch_cost_list=("time",), feed=None):
        if any(c != "time" for c in fetch_cost_list):
            raise ValueError(f"profile_measure: only the 'time' cost is measured (got {list(fetch_cost_list)})")
        import torch
        from .. import static
        from ..static.program import run_program
        dev = "gpu" if device == "gpu" and torch.cuda.is_available() else "cpu"
        exe = static.Executor(static.CUDAPlace(0) if dev == "gpu" else static.CPUPlace())
        ops = main_program.global_block().ops
        if not ops:
            return CostData([], 0.0)
        exe.run(startup_program)
        timer = []
        main_program.__dict__["_op_timer"] = (timer, lambda: _sync(dev))
        try:
            _sync(dev)
            t0 = time.perf_counter()
            run_program(main_program, feed or {}, [])   # every op (no fetch-driven pruning)
            _sync(dev)
            whole = (time.perf_counter() - t0) * 1e3
        finally:
            main_program.__dict__.pop("_op_timer", None)
        top = [ms for blk, _, ms in timer if blk == 0]
        types = [op.type.rsplit(".", 1)[-1] for op in ops]
        return CostData(top, max(whole, sum(top)), types[:len(top)])


class CostModel:
    """reference surface: build a demo program, profile a program, and read the static per-op
    benchmark table"""

    def __init__(self):
        self._static_cost_data = None

    def build_program(self):
        from .. import static, optimizer, mean, enable_static
        enable_static()
        main_program, startup_program = static.Program(), static.Program()
        with static.program_guard(main_program=main_program, startup_program=startup_program):
            data = static.data(name="X", shape=[None, 1], dtype="float32")
            hidden = static.nn.fc(data, 10)
            loss = mean(hidden)
            optimizer.SGD(learning_rate=0.01).minimize(loss)
        return startup_program, main_program

    def profile_measure(self, startup_program, main_program, device="gpu", fetch_cost_list=("time",)):
        import numpy as np
        feed = {"X": np.random.random(size=(10, 1)).astype("float32")} \
            if "X" in main_program.global_block().vars else None
        return _CoreCostModel().profile_measure(main_program, startup_program, device, fetch_cost_list, feed=feed)

    def static_cost_data(self):
        with open(_TABLE) as f:
            self._static_cost_data = json.load(f)
        return self._static_cost_data

    def get_static_op_time(self, op_name, forward=True, dtype="float32"):
        if op_name is None:
            raise ValueError("op_name should not be empty when you want to get static op time")
        if self._static_cost_data is None:
            self.static_cost_data()
        op_cost = {}
        for d in self._static_cost_data:
            if d["op"] == op_name and dtype in d["config"]:
                op_cost["op_time"] = d["paddle_gpu_time"] if forward else d["paddle_gpu_time_backward"]
                op_cost["config"] = d["config"]
        return op_cost
