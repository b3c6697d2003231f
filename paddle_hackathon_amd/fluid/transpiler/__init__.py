"""``fluid.transpiler`` (reference: python/paddle/fluid/transpiler): the 1.x parameter-server
transpiler API. The program is not rewritten: trainers and servers run through the framework's
parameter-server runtime (parallel/ps), which this config object parameterises."""
from __future__ import annotations

__all__ = ["DistributeTranspiler", "DistributeTranspilerConfig", "memory_optimize", "release_memory", "HashName",
           "RoundRobin"]


class DistributeTranspilerConfig:
    def __init__(self):
        self.slice_var_up = True
        self.split_method = None
        self.min_block_size = 8192
        self.sync_mode = True
        self.mode = "pserver"


class HashName:
    def __init__(self, pserver_endpoints):
        self.eps = list(pserver_endpoints)

    def dispatch(self, varlist):
        return [self.eps[hash(v.name) % len(self.eps)] for v in varlist]


class RoundRobin:
    def __init__(self, pserver_endpoints):
        self.eps = list(pserver_endpoints)
        self.i = 0

    def dispatch(self, varlist):
        out = []
        for _ in varlist:
            out.append(self.eps[self.i % len(self.eps)])
            self.i += 1
        return out


class DistributeTranspiler:
    def __init__(self, config=None):
        self.config = config or DistributeTranspilerConfig()

    def transpile(self, trainer_id, program=None, pservers="127.0.0.1:6174", trainers=1, sync_mode=True,
                  startup_program=None, current_endpoint="127.0.0.1:6174"):
        from ..framework import default_main_program
        self.trainer_id, self.trainers = trainer_id, trainers
        self.pserver_endpoints = pservers.split(",") if isinstance(pservers, str) else list(pservers)
        self.origin_program = program or default_main_program()
        self.sync_mode = sync_mode
        self.current_endpoint = current_endpoint

    def get_trainer_program(self, wait_port=True):
        return self.origin_program

    def get_pserver_program(self, endpoint):
        return self.origin_program

    def get_pserver_programs(self, endpoint):
        return self.origin_program, self.origin_program

    def get_startup_program(self, endpoint, pserver_program=None, startup_program=None):
        from ..framework import default_startup_program
        return startup_program or default_startup_program()


def memory_optimize(input_program, skip_opt_set=None, print_log=False, level=0, skip_grads=True):
    """no-op: the executor frees intermediates after their last reader (eager deletion)"""


def release_memory(input_program, skip_opt_set=None):
    """no-op, see memory_optimize"""
