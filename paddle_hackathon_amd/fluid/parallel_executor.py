"""``ParallelExecutor`` (reference: python/paddle/fluid/parallel_executor.py): one process per
GPU here, so it runs the program like ``Executor`` (data parallelism comes from fleet)."""
from ..static.program import Executor

__all__ = ["ParallelExecutor"]


class ParallelExecutor(Executor):
    def __init__(self, use_cuda=True, loss_name=None, main_program=None, share_vars_from=None, exec_strategy=None,
                 build_strategy=None, num_trainers=1, trainer_id=0, scope=None):
        super().__init__()
        self._main = main_program

    def run(self, fetch_list, feed=None, feed_dict=None, return_numpy=True):
        return super().run(self._main, feed=feed or feed_dict, fetch_list=fetch_list, return_numpy=return_numpy)

    @property
    def device_count(self):
        return 1

    def drop_local_exe_scopes(self):
        pass
