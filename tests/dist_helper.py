"""Run a test body in N gloo ranks on CPU (reference pattern: test_dist_base.py /
test_collective_api_base.py launch local trainers and compare results)."""
import os
import socket
import sys
import traceback

import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "PADDLE_TRAINER_ID": str(rank), "PADDLE_TRAINERS_NUM": str(world)})
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        import paddle_hackathon_amd as paddle
        paddle.set_device("cpu")
        paddle.distributed.init_parallel_env(backend="gloo")
        res = fn(rank, world, *args)
        q.put((rank, "ok", res))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        try:
            import torch.distributed as dist
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:
            pass


def run_dist(fn, world=2, args=(), timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, st, val = q.get(timeout=timeout)
            if st != "ok":
                raise AssertionError(f"rank {rank} failed:\n{val}")
            results[rank] = val
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world)]
