"""Role makers (reference: python/paddle/distributed/fleet/base/role_maker.py).

Collective jobs read RANK / WORLD_SIZE (or PADDLE_TRAINER_ID / PADDLE_TRAINERS_NUM). Parameter-server
jobs use the reference's environment: TRAINING_ROLE (TRAINER | PSERVER), PADDLE_PSERVERS_IP_PORT_LIST,
PADDLE_TRAINERS_NUM, PADDLE_TRAINER_ID, and POD_IP + PADDLE_PORT for a server's own endpoint.
"""
import os


class Role:
    WORKER = 1
    SERVER = 2
    HETER_WORKER = 3
    ALL = 4
    COORDINATOR = 5


class PaddleCloudRoleMaker:
    def __init__(self, is_collective=False, **kwargs):
        self._is_collective = is_collective
        self._kwargs = kwargs

    # -- parameter-server environment -------------------------------------------------
    def _get_pserver_endpoints(self):
        eps = os.environ.get("PADDLE_PSERVERS_IP_PORT_LIST", "")
        return [e for e in eps.split(",") if e]

    def _is_ps_mode(self):
        return not self._is_collective and bool(self._get_pserver_endpoints())

    def _training_role(self):
        return os.environ.get("TRAINING_ROLE", "TRAINER").upper()

    def _server_index(self):
        eps = self._get_pserver_endpoints()
        me = f"{os.environ.get('POD_IP', '127.0.0.1')}:{os.environ.get('PADDLE_PORT', '')}"
        if me in eps:
            return eps.index(me)
        port = os.environ.get("PADDLE_PORT")
        for i, e in enumerate(eps):   # any host with our port (single-node launches)
            if port and e.rsplit(":", 1)[1] == port:
                return i
        raise ValueError(f"server endpoint {me} not in PADDLE_PSERVERS_IP_PORT_LIST={eps}")

    def _server_num(self):
        return len(self._get_pserver_endpoints())

    # -- common -------------------------------------------------------------------------
    def _worker_index(self):
        return int(os.environ.get("PADDLE_TRAINER_ID", os.environ.get("RANK", "0")))

    def _worker_num(self):
        return int(os.environ.get("PADDLE_TRAINERS_NUM", os.environ.get("WORLD_SIZE", "1")))

    def _is_worker(self):
        return not self._is_ps_mode() or self._training_role() == "TRAINER"

    def _is_server(self):
        return self._is_ps_mode() and self._training_role() == "PSERVER"

    def _is_first_worker(self):
        return self._is_worker() and self._worker_index() == 0

    def _role_id(self):
        return self._server_index() if self._is_server() else self._worker_index()


class UserDefinedRoleMaker(PaddleCloudRoleMaker):
    def __init__(self, is_collective=False, init_gloo=False, current_id=0, role=Role.WORKER, worker_num=1,
                 server_endpoints=None, **kwargs):
        super().__init__(is_collective)
        self._current_id, self._role, self._wn = current_id, role, worker_num
        self._server_endpoints = list(server_endpoints or [])

    def _get_pserver_endpoints(self):
        return self._server_endpoints

    def _training_role(self):
        return "PSERVER" if self._role == Role.SERVER else "TRAINER"

    def _server_index(self):
        return self._current_id

    def _worker_index(self):
        return self._current_id if self._role == Role.WORKER else 0

    def _worker_num(self):
        return self._wn
