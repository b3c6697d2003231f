"""Process launch (reference: python/paddle/distributed/{spawn.py,launch/main.py},
fleet/launch.py, fleet/elastic/*).

``spawn`` forks one process per device and sets the PADDLE_*/torch rendezvous env.
``launch`` (``python -m paddle_hackathon_amd.distributed.launch --nproc_per_node N script.py``)
starts one process per GPU with a watchdog: if any rank exits non-zero (or stops
heart-beating when ``--heartbeat-timeout`` is set) the whole job is torn down, the
failure-detection role of the reference's elastic/launch controller.
"""
from __future__ import annotations

import argparse
import multiprocessing as mp
import os
import signal
import socket
import subprocess
import sys
import time

__all__ = ["spawn", "launch", "MultiprocessContext"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env_for(rank, world, port, local_rank=None):
    return {
        "RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank if local_rank is None else local_rank),
        "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
        "PADDLE_TRAINER_ID": str(rank), "PADDLE_TRAINERS_NUM": str(world),
        "PADDLE_RANK_IN_NODE": str(rank if local_rank is None else local_rank),
        "PADDLE_TRAINER_ENDPOINTS": ",".join(f"127.0.0.1:{port + 1 + i}" for i in range(world)),
        "PADDLE_CURRENT_ENDPOINT": f"127.0.0.1:{port + 1 + rank}",
        "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
    }


def _worker(func, args, env, q):
    os.environ.update(env)
    try:
        r = func(*args)
        q.put((int(env["RANK"]), "ok", r))
    except Exception as e:  # pragma: no cover - surfaced to the parent
        import traceback
        q.put((int(env["RANK"]), "error", traceback.format_exc()))
        raise


class MultiprocessContext:
    def __init__(self, procs, q):
        self.processes, self._q = procs, q
        self.return_values = {}

    def join(self, timeout=None):
        deadline = None if timeout is None else time.time() + timeout
        errors = []
        while any(p.is_alive() for p in self.processes):
            for p in self.processes:
                if not p.is_alive() and p.exitcode not in (0, None):
                    errors.append(p.exitcode)
            if errors:
                break
            if deadline and time.time() > deadline:
                return False
            time.sleep(0.05)
        while not self._q.empty():
            rank, st, val = self._q.get()
            if st == "error":
                for p in self.processes:
                    if p.is_alive():
                        p.terminate()
                raise RuntimeError(f"rank {rank} failed:\n{val}")
            self.return_values[rank] = val
        for p in self.processes:
            p.join()
            if p.exitcode != 0:
                for o in self.processes:
                    if o.is_alive():
                        o.terminate()
                raise RuntimeError(f"process exited with code {p.exitcode}")
        return True


def spawn(func, args=(), nprocs=-1, join=True, daemon=False, **options):
    if nprocs == -1:
        import torch
        nprocs = max(1, torch.cuda.device_count())
    port = options.get("master_port") or _free_port()
    ctx = mp.get_context(options.get("start_method", "spawn"))
    q = ctx.SimpleQueue()
    procs = []
    for r in range(nprocs):
        p = ctx.Process(target=_worker, args=(func, args, _env_for(r, nprocs, port), q), daemon=daemon)
        p.start()
        procs.append(p)
    c = MultiprocessContext(procs, q)
    if join:
        c.join()
    return c


def launch(argv=None):
    ap = argparse.ArgumentParser("paddle_hackathon_amd.distributed.launch")
    ap.add_argument("--nproc_per_node", "--nproc-per-node", type=int, default=None)
    ap.add_argument("--gpus", "--devices", type=str, default=None)
    ap.add_argument("--master_port", "--master-port", type=int, default=None)
    ap.add_argument("--log_dir", "--log-dir", type=str, default=None)
    ap.add_argument("--heartbeat-timeout", type=float, default=0.0)
    # parameter-server mode (reference: launch --server_num/--servers/--worker_num/--workers)
    ap.add_argument("--server_num", "--server-num", type=int, default=0)
    ap.add_argument("--servers", type=str, default="")
    ap.add_argument("--worker_num", "--worker-num", type=int, default=0)
    ap.add_argument("--workers", type=str, default="")
    # elastic / fault-tolerant mode (reference: launch --elastic_server --job_id --np)
    ap.add_argument("--elastic_server", "--elastic-server", type=str, default=None)
    ap.add_argument("--host_store", action="store_true")
    ap.add_argument("--job_id", "--job-id", type=str, default="default")
    ap.add_argument("--np", type=str, default=None)
    ap.add_argument("--max_restart", "--max-restart", type=int, default=3)
    ap.add_argument("script")
    ap.add_argument("script_args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.server_num or a.servers:
        return _launch_ps(a)
    if a.elastic_server:
        from .elastic import launch_elastic
        a.nproc_per_node = a.nproc_per_node or 1
        a.np = a.np or "1"
        a.heartbeat_timeout = a.heartbeat_timeout or 10.0
        return launch_elastic(a)
    n = a.nproc_per_node or (len(a.gpus.split(",")) if a.gpus else 1)
    port = a.master_port or _free_port()
    procs = []
    hb_dir = None
    if a.heartbeat_timeout > 0:
        import tempfile
        hb_dir = tempfile.mkdtemp(prefix="pha_hb_")
    for r in range(n):
        env = dict(os.environ)
        env.update(_env_for(r, n, port))
        if a.gpus:
            env["FLAGS_selected_gpus"] = a.gpus.split(",")[r]
        if hb_dir:
            env["PHA_HEARTBEAT_FILE"] = os.path.join(hb_dir, f"rank{r}")
        out = None
        if a.log_dir:
            os.makedirs(a.log_dir, exist_ok=True)
            out = open(os.path.join(a.log_dir, f"workerlog.{r}"), "w")
        procs.append(subprocess.Popen([sys.executable, a.script] + a.script_args, env=env, stdout=out,
                                      stderr=subprocess.STDOUT if out else None, start_new_session=True))
    rc = 0
    try:
        while True:
            alive = 0
            for r, p in enumerate(procs):
                c = p.poll()
                if c is None:
                    alive += 1
                    if hb_dir:
                        f = os.path.join(hb_dir, f"rank{r}")
                        if os.path.exists(f) and time.time() - os.path.getmtime(f) > a.heartbeat_timeout:
                            print(f"[launch] rank {r} heartbeat lost; terminating job", file=sys.stderr)
                            rc = 1
                            raise KeyboardInterrupt
                elif c != 0:
                    print(f"[launch] rank {r} exited with {c}; terminating job", file=sys.stderr)
                    rc = c
                    raise KeyboardInterrupt
            if alive == 0:
                break
            time.sleep(0.2)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
        rc = rc or 1
    return rc


def _launch_ps(a):
    """Parameter-server job on this node: server processes (TRAINING_ROLE=PSERVER) and trainer
    processes (TRAINING_ROLE=TRAINER) with the reference's PADDLE_* environment. Any failing
    trainer ends the job; once every trainer has exited the servers get 30 s to stop."""
    servers = [e for e in a.servers.split(",") if e] or [f"127.0.0.1:{_free_port()}" for _ in range(a.server_num)]
    nw = a.worker_num or len([w for w in a.workers.split(",") if w]) or a.nproc_per_node or 1
    base = dict(os.environ)
    base.update({"PADDLE_PSERVERS_IP_PORT_LIST": ",".join(servers), "PADDLE_TRAINERS_NUM": str(nw)})
    log = (lambda name: open(os.path.join(a.log_dir, name), "w")) if a.log_dir else (lambda name: None)
    if a.log_dir:
        os.makedirs(a.log_dir, exist_ok=True)

    def start(env, name):
        out = log(name)
        return subprocess.Popen([sys.executable, a.script] + a.script_args, env=env, stdout=out,
                                stderr=subprocess.STDOUT if out else None, start_new_session=True)

    srv, trn = [], []
    for i, ep in enumerate(servers):
        host, port = ep.rsplit(":", 1)
        env = dict(base, TRAINING_ROLE="PSERVER", POD_IP=host, PADDLE_PORT=port)
        srv.append(start(env, f"serverlog.{i}"))
    for r in range(nw):
        env = dict(base, TRAINING_ROLE="TRAINER", PADDLE_TRAINER_ID=str(r), POD_IP="127.0.0.1",
                   PADDLE_PORT=str(_free_port()))
        trn.append(start(env, f"workerlog.{r}"))
    rc = 0
    try:
        while any(p.poll() is None for p in trn):
            for r, p in enumerate(trn):
                c = p.poll()
                if c not in (None, 0):
                    print(f"[launch] trainer {r} exited with {c}; terminating job", file=sys.stderr)
                    rc = c
                    raise KeyboardInterrupt
            for i, p in enumerate(srv):
                if p.poll() not in (None, 0):
                    print(f"[launch] server {i} exited with {p.returncode}; terminating job", file=sys.stderr)
                    rc = p.returncode
                    raise KeyboardInterrupt
            time.sleep(0.2)
        for r, p in enumerate(trn):   # the last trainers may have exited together, some failing
            if p.returncode not in (None, 0):
                print(f"[launch] trainer {r} exited with {p.returncode}", file=sys.stderr)
                rc = rc or p.returncode
        deadline = time.time() + 30
        while any(p.poll() is None for p in srv) and time.time() < deadline:
            time.sleep(0.2)
    except KeyboardInterrupt:
        rc = rc or 1
    for p in srv + trn:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    for p in srv + trn:
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
    return rc


def heartbeat():
    """Call periodically from a training loop launched with --heartbeat-timeout."""
    f = os.environ.get("PHA_HEARTBEAT_FILE")
    if f:
        with open(f, "a"):
            os.utime(f, None)


if __name__ == "__main__":
    sys.exit(launch())
