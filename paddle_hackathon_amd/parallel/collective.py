"""Collective communication (reference: python/paddle/distributed/collective.py,
python/paddle/distributed/parallel.py, paddle/fluid/distributed/collective/ProcessGroupNCCL.cc).

One process per GPU. ``torch.distributed`` with backend ``"nccl"`` *is* RCCL on
ROCm (collectives over xGMI between MI355X GPUs); ``"gloo"`` is used on CPU.
Groups are Paddle ``Group`` objects wrapping a torch ProcessGroup.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

from ..framework.core import Tensor, _wrap, _unwrap

__all__ = ["ReduceOp", "Group", "ParallelEnv", "init_parallel_env", "get_rank", "get_world_size", "is_initialized",
           "new_group", "get_group", "all_reduce", "broadcast", "reduce", "all_gather", "all_gather_object",
           "scatter", "alltoall", "alltoall_single", "reduce_scatter", "send", "recv", "isend", "irecv", "barrier",
           "wait", "destroy_process_group", "get_backend", "stream", "batch_isend_irecv", "P2POp",
           "broadcast_object_list"]


class ReduceOp:
    SUM = 0
    MAX = 1
    MIN = 2
    PROD = 3
    AVG = 4


_TORCH_OP = {ReduceOp.SUM: dist.ReduceOp.SUM, ReduceOp.MAX: dist.ReduceOp.MAX, ReduceOp.MIN: dist.ReduceOp.MIN,
             ReduceOp.PROD: dist.ReduceOp.PRODUCT}


class Group:
    def __init__(self, rank_in_group, id, ranks, pg=None, name=None):
        self.rank = rank_in_group
        self.id = id
        self.ranks = list(ranks)
        self.nranks = len(ranks)
        self.pg = pg
        self.name = name

    @property
    def world_size(self):
        return self.nranks

    @property
    def process_group(self):
        return self.pg

    def is_member(self):
        return self.rank >= 0

    def get_group_rank(self, rank):
        return self.ranks.index(rank) if rank in self.ranks else -1

    def __repr__(self):
        return f"Group(rank={self.rank}, nranks={self.nranks}, id={self.id}, ranks={self.ranks})"


_groups = {}
_global_group = None
_backend = None


def _env_int(*names, default=0):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return int(v)
    return default


class ParallelEnv:
    """Trainer environment (reference: python/paddle/fluid/dygraph/parallel.py:ParallelEnv)."""

    def __init__(self):
        self._rank = _env_int("PADDLE_TRAINER_ID", "RANK", default=0)
        self._world_size = _env_int("PADDLE_TRAINERS_NUM", "WORLD_SIZE", default=1)
        self._local_rank = _env_int("PADDLE_RANK_IN_NODE", "LOCAL_RANK", default=self._rank)
        self._device_id = _env_int("FLAGS_selected_gpus", default=self._local_rank) if "FLAGS_selected_gpus" in os.environ else self._local_rank
        eps = os.environ.get("PADDLE_TRAINER_ENDPOINTS", "")
        self._trainer_endpoints = eps.split(",") if eps else []
        self._current_endpoint = os.environ.get("PADDLE_CURRENT_ENDPOINT", "")
        self._nrings = _env_int("FLAGS_nccl_nrings", default=1)

    @property
    def rank(self):
        return self._rank

    @property
    def world_size(self):
        return self._world_size

    @property
    def device_id(self):
        return self._device_id

    @property
    def local_rank(self):
        return self._local_rank

    @property
    def current_endpoint(self):
        return self._current_endpoint

    @property
    def trainer_endpoints(self):
        return self._trainer_endpoints

    @property
    def nrings(self):
        return self._nrings

    nranks = world_size
    dev_id = device_id


def is_initialized():
    return dist.is_available() and dist.is_initialized()


def init_parallel_env(backend=None, timeout_s=1800):
    """Initialise the default group. Backend: RCCL (``nccl``) when a GPU is visible, else gloo."""
    global _global_group, _backend
    if is_initialized():
        if _global_group is None:
            _make_global()
        return _global_group
    env = ParallelEnv()
    os.environ.setdefault("MASTER_ADDR", os.environ.get("PADDLE_MASTER_ADDR", "127.0.0.1"))
    os.environ.setdefault("MASTER_PORT", os.environ.get("PADDLE_MASTER_PORT", "29500"))
    os.environ.setdefault("RANK", str(env.rank))
    os.environ.setdefault("WORLD_SIZE", str(env.world_size))
    if backend is None:   # PHA_DIST_BACKEND=gloo: host collectives even with GPUs (multi-rank rehearsal on one GPU)
        backend = os.environ.get("PHA_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend in ("nccl", "rccl") and torch.cuda.is_available():
        torch.cuda.set_device(env.device_id % max(1, torch.cuda.device_count()))
        from ..framework import core
        core.set_device(f"gpu:{env.device_id % max(1, torch.cuda.device_count())}")
        backend = "nccl"
        dev_id = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group("nccl", rank=env.rank, world_size=env.world_size,
                                timeout=datetime.timedelta(seconds=timeout_s), device_id=dev_id)
    else:
        backend = "gloo"
        dist.init_process_group("gloo", rank=env.rank, world_size=env.world_size,
                                timeout=datetime.timedelta(seconds=timeout_s))
    _backend = backend
    _make_global()
    return _global_group


def _make_global():
    global _global_group
    ws = dist.get_world_size()
    _global_group = Group(dist.get_rank(), 0, list(range(ws)), dist.group.WORLD, "_default_pg")
    _groups[0] = _global_group


def get_backend(group=None):
    return _backend or (dist.get_backend() if is_initialized() else None)


def destroy_process_group(group=None):
    global _global_group
    if group is None:
        if is_initialized():
            dist.destroy_process_group()
        _groups.clear()
        _global_group = None
    else:
        _groups.pop(group.id, None)


def get_rank(group=None):
    if group is not None:
        return group.rank
    if is_initialized():
        return dist.get_rank()
    return _env_int("PADDLE_TRAINER_ID", "RANK", default=0)


def get_world_size(group=None):
    if group is not None:
        return group.nranks
    if is_initialized():
        return dist.get_world_size()
    return _env_int("PADDLE_TRAINERS_NUM", "WORLD_SIZE", default=1)


_next_gid = [1]


def new_group(ranks=None, backend=None, timeout=None):
    """Every rank must call new_group with the same ranks (torch.distributed semantics)."""
    if not is_initialized():
        init_parallel_env()
    ws = dist.get_world_size()
    ranks = sorted(ranks) if ranks is not None else list(range(ws))
    if ranks == list(range(ws)):
        pg = dist.group.WORLD
    else:
        pg = dist.new_group(ranks, backend=None if backend in (None, "nccl", "rccl") else backend)
    me = dist.get_rank()
    gid = _next_gid[0]
    _next_gid[0] += 1
    g = Group(ranks.index(me) if me in ranks else -1, gid, ranks, pg if me in ranks else None)
    _groups[gid] = g
    return g


def get_group(id=0):
    return _groups.get(id)


def _resolve_group(group):
    if group is None:
        return dist.group.WORLD
    if isinstance(group, Group):
        return group.pg
    return group


def _t(x):
    return x._t if isinstance(x, Tensor) else x


class _Task:
    def __init__(self, work, post=None):
        self._work, self._post = work, post

    def wait(self):
        if self._work is not None:
            self._work.wait()
        if self._post is not None:
            self._post()
            self._post = None
        return True

    def is_completed(self):
        return self._work is None or self._work.is_completed()


def _nranks(group):
    return group.nranks if isinstance(group, Group) else dist.get_world_size(_resolve_group(group))


def all_reduce(tensor, op=ReduceOp.SUM, group=None, use_calc_stream=True, sync_op=True):
    if isinstance(group, Group) and not group.is_member():
        return None
    t = _t(tensor)
    pg = _resolve_group(group)
    post = None
    if op == ReduceOp.AVG:
        if get_backend() == "nccl":
            top = dist.ReduceOp.AVG
        else:
            top = dist.ReduceOp.SUM
            n = _nranks(group)
            post = lambda: t.div_(n)
    else:
        top = _TORCH_OP[op]
    work = dist.all_reduce(t, op=top, group=pg, async_op=not sync_op)
    if sync_op:
        if post:
            post()
        return None
    return _Task(work, post)


def broadcast(tensor, src, group=None, use_calc_stream=True, sync_op=True):
    if isinstance(group, Group) and not group.is_member():
        return None
    work = dist.broadcast(_t(tensor), src=src, group=_resolve_group(group), async_op=not sync_op)
    return None if sync_op else _Task(work)


def broadcast_object_list(object_list, src, group=None):
    dist.broadcast_object_list(object_list, src=src, group=_resolve_group(group))


def reduce(tensor, dst, op=ReduceOp.SUM, group=None, use_calc_stream=True, sync_op=True):
    t = _t(tensor)
    if op == ReduceOp.AVG:
        work = dist.reduce(t, dst=dst, op=dist.ReduceOp.SUM, group=_resolve_group(group), async_op=not sync_op)
        if sync_op and get_rank() == dst:
            t.div_(_nranks(group))
        return None if sync_op else _Task(work)
    work = dist.reduce(t, dst=dst, op=_TORCH_OP[op], group=_resolve_group(group), async_op=not sync_op)
    return None if sync_op else _Task(work)


def all_gather(tensor_list, tensor, group=None, use_calc_stream=True, sync_op=True):
    t = _t(tensor)
    n = _nranks(group)
    outs = [torch.empty_like(t) for _ in range(n)]
    work = dist.all_gather(outs, t.contiguous(), group=_resolve_group(group), async_op=not sync_op)

    def fill():
        tensor_list.clear()
        tensor_list.extend(_wrap(o) for o in outs)
    if sync_op:
        fill()
        return None
    return _Task(work, fill)


def all_gather_object(object_list, obj, group=None):
    n = _nranks(group)
    out = [None] * n
    dist.all_gather_object(out, obj, group=_resolve_group(group))
    object_list.clear()
    object_list.extend(out)


def scatter(tensor, tensor_list=None, src=0, group=None, use_calc_stream=True, sync_op=True):
    t = _t(tensor)
    pg = _resolve_group(group)
    me = dist.get_rank()
    gsrc = src
    lst = [_t(x).contiguous() for x in tensor_list] if (tensor_list is not None and me == gsrc) else None
    work = dist.scatter(t, lst, src=src, group=pg, async_op=not sync_op)
    return None if sync_op else _Task(work)


def alltoall(in_tensor_list, out_tensor_list, group=None, use_calc_stream=True, sync_op=True):
    ins = [_t(x).contiguous() for x in in_tensor_list]
    outs = [torch.empty_like(i) for i in ins]
    if get_backend() == "gloo":
        # gloo has no all_to_all: emulate with scatter from every rank
        n = len(ins)
        pg = _resolve_group(group)
        for src in range(n):
            gsrc = group.ranks[src] if isinstance(group, Group) else src
            dist.scatter(outs[src], ins if dist.get_rank() == gsrc else None, src=gsrc, group=pg)
        work = None
    else:
        work = dist.all_to_all(outs, ins, group=_resolve_group(group), async_op=not sync_op)

    def fill():
        out_tensor_list.clear()
        out_tensor_list.extend(_wrap(o) for o in outs)
    if sync_op or work is None:
        fill()
        return None
    return _Task(work, fill)


def alltoall_single(in_tensor, out_tensor, in_split_sizes=None, out_split_sizes=None, group=None,
                    use_calc_stream=True, sync_op=True):
    i, o = _t(in_tensor), _t(out_tensor)
    if get_backend() == "gloo":
        n = _nranks(group)
        ins = list(torch.split(i, in_split_sizes or [i.shape[0] // n] * n))
        outs = []
        alltoall([_wrap(x) for x in ins], outs, group)
        o.copy_(torch.cat([x._t for x in outs]))
        return None
    work = dist.all_to_all_single(o, i, out_split_sizes, in_split_sizes, group=_resolve_group(group), async_op=not sync_op)
    return None if sync_op else _Task(work)


def reduce_scatter(tensor, tensor_list, op=ReduceOp.SUM, group=None, use_calc_stream=True, sync_op=True):
    t = _t(tensor)
    lst = [_t(x).contiguous() for x in tensor_list]
    if get_backend() == "gloo":
        full = torch.stack(lst)
        dist.all_reduce(full, op=_TORCH_OP[op if op != ReduceOp.AVG else ReduceOp.SUM], group=_resolve_group(group))
        me = group.rank if isinstance(group, Group) else dist.get_rank()
        t.copy_(full[me])
        if op == ReduceOp.AVG:
            t.div_(len(lst))
        return None
    top = dist.ReduceOp.AVG if op == ReduceOp.AVG else _TORCH_OP[op]
    work = dist.reduce_scatter(t, lst, op=top, group=_resolve_group(group), async_op=not sync_op)
    return None if sync_op else _Task(work)


def _global_peer(peer, group):
    return group.ranks[peer] if isinstance(group, Group) else peer


def send(tensor, dst=0, group=None, use_calc_stream=True, sync_op=True):
    if sync_op:
        dist.send(_t(tensor).contiguous(), _global_peer(dst, group), group=_resolve_group(group))
        return None
    return _Task(dist.isend(_t(tensor).contiguous(), _global_peer(dst, group), group=_resolve_group(group)))


def recv(tensor, src=0, group=None, use_calc_stream=True, sync_op=True):
    if sync_op:
        dist.recv(_t(tensor), _global_peer(src, group), group=_resolve_group(group))
        return None
    return _Task(dist.irecv(_t(tensor), _global_peer(src, group), group=_resolve_group(group)))


def isend(tensor, dst, group=None):
    return send(tensor, dst, group, sync_op=False)


def irecv(tensor, src=None, group=None):
    return recv(tensor, src, group, sync_op=False)


class P2POp:
    def __init__(self, op, tensor, peer, group=None):
        self.op, self.tensor, self.peer, self.group = op, tensor, peer, group


def batch_isend_irecv(p2p_op_list):
    ops = []
    for p in p2p_op_list:
        f = dist.isend if p.op in (isend, dist.isend) else dist.irecv
        ops.append(dist.P2POp(f, _t(p.tensor), _global_peer(p.peer, p.group), _resolve_group(p.group)))
    works = dist.batch_isend_irecv(ops)
    return [_Task(w) for w in works]


def barrier(group=None):
    if not is_initialized():
        return
    pg = _resolve_group(group)
    if get_backend() == "nccl":
        dist.barrier(group=pg, device_ids=[torch.cuda.current_device()])
    else:
        dist.barrier(group=pg)


def wait(tensor, group=None, use_calc_stream=True):
    if torch.cuda.is_available():
        torch.cuda.current_stream().synchronize()


class stream:
    """paddle.distributed.stream.* variants (explicit comm-stream control) map to async collectives."""

    @staticmethod
    def all_reduce(tensor, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False):
        return all_reduce(tensor, op, group, use_calc_stream, sync_op)

    @staticmethod
    def all_gather(tensor_or_tensor_list, tensor, group=None, sync_op=True, use_calc_stream=False):
        return all_gather(tensor_or_tensor_list, tensor, group, use_calc_stream, sync_op)

    @staticmethod
    def reduce_scatter(tensor, tensor_list, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False):
        return reduce_scatter(tensor, tensor_list, op, group, use_calc_stream, sync_op)
