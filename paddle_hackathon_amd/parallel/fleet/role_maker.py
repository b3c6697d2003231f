"""Role makers (reference: python/paddle/distributed/fleet/base/role_maker.py). Collective mode."""
import os


class Role:
    WORKER = 1
    SERVER = 2
    HETER_WORKER = 3
    ALL = 4


class PaddleCloudRoleMaker:
    def __init__(self, is_collective=False, **kwargs):
        self._is_collective = is_collective

    def _worker_index(self):
        return int(os.environ.get("PADDLE_TRAINER_ID", os.environ.get("RANK", "0")))

    def _worker_num(self):
        return int(os.environ.get("PADDLE_TRAINERS_NUM", os.environ.get("WORLD_SIZE", "1")))

    def _is_worker(self):
        return True

    def _is_server(self):
        return False

    def _role_id(self):
        return self._worker_index()


class UserDefinedRoleMaker(PaddleCloudRoleMaker):
    def __init__(self, is_collective=False, init_gloo=False, current_id=0, role=Role.WORKER, worker_num=1,
                 server_endpoints=None, **kwargs):
        super().__init__(is_collective)
        self._current_id, self._role, self._wn = current_id, role, worker_num

    def _worker_index(self):
        return self._current_id

    def _worker_num(self):
        return self._wn
