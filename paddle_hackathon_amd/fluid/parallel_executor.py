"""``ParallelExecutor`` (reference: python/paddle/fluid/parallel_executor.py). One process drives
one MI355X, so the data parallelism is over the job's ranks: with ``num_trainers`` > 1 (or an
initialised process group of more than one rank) the program's gradients are all-reduced before
its optimizer ops (static/program.py data_parallel_program, the bucketed overlapped RCCL all-reduce
of the static fleet DP pass); ``device_count`` is the number of ranks."""
import os

from ..static.program import Executor, CompiledProgram, default_main_program

__all__ = ["ParallelExecutor"]


class ParallelExecutor(Executor):
    def __init__(self, use_cuda=True, loss_name=None, main_program=None, share_vars_from=None, exec_strategy=None,
                 build_strategy=None, num_trainers=1, trainer_id=0, scope=None):
        super().__init__()
        import torch.distributed as tdist
        self._main = main_program if main_program is not None else default_main_program()
        self._scope = scope
        initialised = tdist.is_available() and tdist.is_initialized()
        if num_trainers > 1 and not initialised:
            raise RuntimeError(f"ParallelExecutor(num_trainers={num_trainers}): initialise the process group first "
                               "(paddle.distributed.init_parallel_env / fleet.init), one process per GPU")
        self._world = tdist.get_world_size() if initialised else 1
        if num_trainers > 1 and self._world != num_trainers:
            raise ValueError(f"num_trainers={num_trainers} but the process group has {self._world} ranks")
        if self._world > 1:
            os.environ.setdefault("PADDLE_TRAINERS_NUM", str(self._world))
            self._compiled = CompiledProgram(self._main, build_strategy).with_data_parallel(loss_name)
        else:
            self._compiled = None

    def run(self, fetch_list, feed=None, feed_dict=None, return_numpy=True):
        return super().run(self._compiled or self._main, feed=feed or feed_dict, fetch_list=fetch_list,
                           return_numpy=return_numpy, scope=self._scope)

    @property
    def device_count(self):
        return self._world

    def drop_local_exe_scopes(self):
        pass
