"""``fluid.transpiler`` (reference: python/paddle/fluid/transpiler): the 1.x parameter-server /
collective transpiler (distribute_transpiler.py) and the memory-optimisation entry points."""
from __future__ import annotations

from .distribute_transpiler import (DistributeTranspiler, DistributeTranspilerConfig, HashName, RoundRobin,  # noqa: F401
                                    slice_variable)

__all__ = ["DistributeTranspiler", "DistributeTranspilerConfig", "memory_optimize", "release_memory", "HashName",
           "RoundRobin"]


def memory_optimize(input_program, skip_opt_set=None, print_log=False, level=0, skip_grads=True):
    """no-op: the executor frees intermediates after their last reader (eager deletion,
    static/program.py _gc_plan) and plans a static arena for the rest"""


def release_memory(input_program, skip_opt_set=None):
    """no-op, see memory_optimize"""
